#!/usr/bin/env python3
"""Headline benchmark: env-steps/s of the full PPO rollout (BASELINE.json configs[2]:
4096 envs x 16 UAVs x 32 targets, transformer policy + env step on each MI355X).

One timed "step" = one rollout iteration per rank: T (=64) x {fused policy forward (fp32-accurate MFMA) ->
on-device sample -> fused env step (fp64)} over E envs -- all T steps in ONE k_rollout_steps launch
(--per-step-launch: one launch per step) -- a bootstrap value pass, GAE + advantage normalisation,
and with N > 1 GPUs the all-gather of the trajectories: pipelined peer-to-peer copies
beside the next rollout, or one RCCL all-gather after each rollout (--rccl-gather / fallback).
value = E * T * K * N / max-over-ranks wall time. Inputs (scenes, windows) are resident in HBM.

Also reported (same JSON line):
  roofline      dominant kernel = k_rollout_steps (per-step figures: its launch / T); peak = the MFMA
                peak of its FLOP mix (the encoder GEMMs as fp32-accurate split products on the f16
                cores at 16/3 x the f32 MFMA rate, embeddings and heads on the f32 MFMA);
                achieved = ALGORITHMIC FLOP per step (2,446,208 FLOP/sample, the
                last-token-pruned forward of one window) x E / its HIP-event duration per step in the
                last timed iteration; traffic = PMC bytes per step (profiles/rNN_pmc.json). The rollout's
                window-row ring reuses layer-0 Q/K/V of rows 0-3 from earlier steps, so it EXECUTES
                1,790,848 FLOP/sample; that rate is reported beside it (executed_*)
  env_roofline  the env step inside k_rollout_steps against HBM, algorithmic 24*M + 490 B per
                env-step: its time = the per-step time above x its share of the step's
                cycles (s_memtime phase stamps of the TRACE build, scripts/env_phase.py, run as a
                child process); traffic = PMC bytes per step it adds (product build minus a build
                with the env step compiled out, profiles/rNN_env_share.json)
  env_fused     env-only multi-step launches, T = 256 (K2r omega = 0 replay / K2): BASELINE configs[1]
                (1024 envs x 8 x 16) and the headline shape, env-steps/s and algorithmic GB/s; and
                BASELINE configs[4]'s per-GPU shard (8192 envs x 64 x 128, fp16 obs, T = 64)
  score_pairs   K1 (LDS-tiled pair scoring) over 8192 fresh 64 x 128 scenes (configs[4])
  ppo_samples_per_s  one PPO update (5 epochs) over the iteration's batch on the HIP training step
                (uavhip_ppo_step) at minibatch 4096 per GPU; N > 1: over the all-gathered batch, data
                parallel (each rank a 1/N slice of every global minibatch, RCCL all-reduce of loss sums
                and gradients)
  ppo_samples_per_s_mb64  the same update at the reference's minibatch 64 (parity mode: the
                reference's optimizer trajectory) over 16,384 of the iteration's transitions, N = 1
  dropin_loop   the reference's own loop (main_train.py:79-146) at E = 1 through the drop-in UAVEnv /
                PPOAgent (30 x 10 and the headline shape): env-steps/s, update() samples/s at minibatch
                64, host syncs per step; the CPU port of the same loop beside it (oracle/cpu_loop_bench.py)
  cpu_baseline  the CPU port (C oracle env.step + torch-CPU fp32 policy + numpy GAE) on host cores,
                rank 0 at N = 1 only, bounded sample
  cpu_env_baseline  UAVEnv.step alone (C oracle, reference algorithm) on all host cores (one process
                per core, <= 16), 10 s
Launch for N > 1: `python bench.py --gpus N` starts the N rank processes itself (launch_plan /
spawn_ranks: RANK / LOCAL_RANK / WORLD_SIZE, MASTER_ADDR 127.0.0.1), or under a launcher
(python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N), whose WORLD_SIZE must equal N.
The N > 1 exchange (collective all-gather after each rollout, or pipelined peer copies beside the next
rollout) is chosen by a short untimed measurement of both; the line reports both (exchange.calibration).
"""
import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "target-allocation-ppo-transformer_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

POLICY_FLOP_PER_SAMPLE = 2_446_208  # full-window forward (last-token pruned), DESIGN.md 4
# the rollout's window-row path (uavhip_policy_forward_rows) forms layer-0 Q|K|V of the new row
# only: minus 4 rows x (actor K,V 256 + critic Q,K,V 384) x 128 x 2 FLOP
ROWS_FLOP_PER_SAMPLE = POLICY_FLOP_PER_SAMPLE - 4 * (256 + 384) * 128 * 2  # 1,790,848
# of these, every encoder GEMM runs as split products on the f16 matrix cores (3 x
# v_mfma_f32_16x16x32_f16 per fp32-accurate 16 x 16 x 32 block), per 16-sample workgroup:
# the critic's layer 0 out-projection + FFN over 80 tokens, its layer-1 K / V over 80 tokens and Q over
# 16, the out-projection + FFN of both pruned top layers over 16 tokens, and -- on the window-row
# ring -- the new row's layer-0 Q | K | V of both trunks (16 tokens). The embeddings and heads stay on
# the f32 MFMA.
_SPLIT_WG = ((128 + 2 * 256) * 128 * 2 * 80 + 256 * 128 * 2 * 80 + 128 * 128 * 2 * 16
             + 2 * (128 + 2 * 256) * 128 * 2 * 16)
SPLIT_FLOP_PER_SAMPLE = _SPLIT_WG // 16                                         # full window: 1,507,328
SPLIT_FLOP_PER_SAMPLE_ROWS = (_SPLIT_WG + 2 * 384 * 128 * 2 * 16) // 16         # ring: 1,703,936
MFMA_SPLIT_PEAK_TFLOPS = 157.3 * 16 / 3  # fp32-equivalent: f16 MFMA (16x the f32 rate) / 3 products
TRAIN_FLOP_PER_SAMPLE_EPOCH = 3 * 4_040_000  # training ~ 3 x dense forward
TRAIN_EXEC_FLOP_PER_SAMPLE_EPOCH = 7_460_000  # pruned forward + dX + dW
# where that work runs: the forward's encoder GEMMs and the encoder layers' input
# gradients (dX: K6 / K7 on the transposed split copies) as two-plane split products (3 f16 MFMAs per
# block), the weight gradients (k_wgrad) as three-plane split products (6 f16 MFMAs per block), the
# embeddings and heads on the f32 MFMA
TRAIN_FWD_SPLIT_FLOP = 2_446_208 - 2 * 80 * 128 * 16 * 2 // 16 - 2 * 64 * 128 * 2  # 2,389,248
# dX per sample: the critic's full layer 0 over its 5 tokens (Win^T 384, Wo^T 128, W1^T / W2^T 256
# each, x 128 x 2) + the two pruned top layers (Wo^T / W1^T / W2^T on token 4, Win^T's dq on token 4
# and dk | dv on all 5)
TRAIN_DX_SPLIT_FLOP = 5 * (384 + 128 + 256 + 256) * 128 * 2 + 2 * ((128 + 256 + 256 + 128) + 5 * 256) * 128 * 2
TRAIN_WGRAD_FLOP = 2_390_000
MFMA_SPLIT3_PEAK_TFLOPS = 157.3 * 16 / 6
MFMA_F32_PEAK_TFLOPS = 157.3          # MI355X_MICROARCH.md: fp32 MFMA = vector peak
HBM_PEAK_GBS = 8000.0


def _kernel_base(name):
    """Kernel name without namespaces and template arguments: 'uavhip::pol::k_rollout_steps<1>' ->
    'k_rollout_steps' (rocprofv3 reports the demangled template instance)."""
    import re
    return re.sub(r"<.*>$", "", name).split("::")[-1].strip()


def _round_files(pattern, exclude=None):
    """profiles/<tag>_... files in round order: tags rNN<suffix> sort by round, then suffix length, then
    suffix (r05t < r05aa: a measurement set tagged after r05z), so files[-1] is the newest set."""
    import glob
    files = [f for f in glob.glob(os.path.join(ROOT, "profiles", pattern)) if not (exclude and exclude in f)]

    def key(f):
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, os.path.basename(f))
    return sorted(files, key=key)


def profiled_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/rNN_pmc.json, written by scripts/summarize_profile.py from separate rocprofv3
    --pmc FETCH_SIZE / WRITE_SIZE passes of this benchmark; FETCH doubled per the gfx950 note).
    Matched on the exact name first, then on the name without namespaces / template arguments
    (a template kernel such as k_rollout_steps<1> is reported with its arguments)."""
    files = _round_files("r*_pmc.json", exclude="train")
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    pmc = {k: v for k, v in d.get("pmc", {}).items() if "hbm_bytes_per_launch" in v}
    for k, v in pmc.items():
        if k.replace("uavhip::pol::", "").replace("uavhip::", "") == kernel:
            return v["hbm_bytes_per_launch"], os.path.basename(files[-1])
    hits = [v for k, v in pmc.items() if _kernel_base(k) == _kernel_base(kernel)]
    if len(hits) == 1:
        return hits[0]["hbm_bytes_per_launch"], os.path.basename(files[-1])
    return None, None


def profiled_kernel_time(kernel):
    """rocprofv3 --kernel-trace --stats durations of `kernel` from the newest committed profile summary
    (profiles/rNN_pmc.json kernel_stats, scripts/profile.sh in the same gpurun lease as a bench run of
    the same code): the average over every launch of the profiled bench run (warm-up and capture
    launches included) and over its timed launches only (summarize_profile.py TIMED_LAUNCHES)."""
    files = _round_files("r*_pmc.json", exclude="train")
    if not files:
        return None
    ks = json.load(open(files[-1])).get("kernel_stats", {})
    for k, v in ks.items():
        if _kernel_base(k) == _kernel_base(kernel):
            return dict(v, kernel=k, source=os.path.basename(files[-1]))
    return None


def env_differential(args, pairs=2):
    """The env step's time inside k_rollout_steps, live on this box: scripts/rollout_run.py as a child
    process (its own GPU context) on the product library and on the build with the env step
    compiled out (libuavhip_noenv.so, make NOENV=1; profiling only, wrong results), alternated
    `pairs` times; each run reports the median HIP-event time per step of its k_rollout_steps
    launches. Returns ({product_ms, noenv_ms, env_ms (medians per step)}, None) or (None, reason)."""
    import subprocess
    libdir = os.path.join(ROOT, "target-allocation-ppo-transformer_amd", "uavhip")
    libs = {"product": os.path.join(libdir, "libuavhip.so"), "noenv": os.path.join(libdir, "libuavhip_noenv.so")}
    if not os.path.exists(libs["noenv"]):
        return None, "no NOENV build (libuavhip_noenv.so)"
    got = {"product": [], "noenv": []}
    try:
        for _ in range(pairs):
            for b in ("product", "noenv"):
                env = dict(os.environ, UAVHIP_LIB=libs[b], E=str(args.envs), N=str(args.uavs), M=str(args.targets),
                           T=str(args.horizon), ITERS="6")
                out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rollout_run.py")], env=env,
                                     capture_output=True, text=True, timeout=300)
                if out.returncode != 0:
                    return None, f"rollout_run.py ({b}) failed: " + out.stderr[-300:]
                got[b].append(json.loads(out.stdout.strip().splitlines()[-1])["step_ms"])
    except Exception as exc:
        return None, repr(exc)
    prod, noenv = float(np.median(got["product"])), float(np.median(got["noenv"]))
    return {"product_ms": prod, "noenv_ms": noenv, "env_ms": prod - noenv, "runs": got}, None


def env_phase_share(args):
    """The env step's share of a k_rollout_steps step from the TRACE build's phase stamps
    (scripts/env_phase.py in a child process: its own GPU context, the product library stays
    loaded here). None (with the reason) when the TRACE build is absent or the probe fails."""
    import subprocess
    lib = os.path.join(ROOT, "target-allocation-ppo-transformer_amd", "uavhip", "libuavhip_trace.so")
    if not os.path.exists(lib):
        return None, "no TRACE build (libuavhip_trace.so)"
    env = dict(os.environ, UAVHIP_LIB=lib, E=str(args.envs), N=str(args.uavs), M=str(args.targets),
               T=str(args.horizon))
    try:
        out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "env_phase.py")], env=env,
                             capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            return None, "env_phase.py failed: " + out.stderr[-300:]
        return json.loads(out.stdout.strip().splitlines()[-1]), None
    except Exception as exc:
        return None, repr(exc)


def env_share_traffic():
    """HBM bytes per env step inside k_rollout_steps (per step of the launch, all E envs) from the
    newest profiles/rNN_env_share.json (scripts/profile_env_share.sh: PMC FETCH/WRITE passes of the
    product build and of a build with the env step compiled out; the difference), with the
    profiled time differential of the same runs."""
    files = _round_files("r*_env_share.json")
    if not files:
        return None, None, None
    d = json.load(open(files[-1]))
    return d.get("env_bytes_per_step"), os.path.basename(files[-1]), d.get("env_ns_per_step")


def env_counters(kernel, grid=None):
    """The VALU side and the PMC traffic of an env kernel (K1 / K2 / K2g / K2r) from the newest
    profiles/rNN_env_counters.json (scripts/profile_env_counters.sh + summarize_env_counters.py, the
    same shapes as the bench's env legs): fp64 FLOP fraction of the 78.6 TFLOP/s fp64 vector peak,
    VALU busy share of SIMD cycles, HBM bytes per launch (FETCH x 2 + WRITE). Matched by kernel name
    without template arguments AND launch grid (threads) when the file keys its entries "name@grid"
    (one template instance serves several shapes)."""
    files = _round_files("r*_env_counters.json")
    if not files:
        return None
    ks = json.load(open(files[-1]))["kernels"]
    k = None
    for name, v in ks.items():
        base, _, g = name.partition("@")
        if _kernel_base(base) == _kernel_base(kernel) and (not g or grid is None or int(g) == int(grid)):
            k, kernel = v, name
            break
    if k is None:
        return None
    keep = ("avg_ns", "fp64_frac", "fp64_tflops", "valu_busy", "hbm_bytes_per_launch", "valu_insts", "salu_insts")
    return dict({a: k[a] for a in keep}, kernel=kernel, source=os.path.basename(files[-1]),
                hbm_frac=k["hbm_bytes_per_launch"] / (k["avg_ns"] * 1e-9) / 1e9 / HBM_PEAK_GBS)


L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md: L2, 8 XCDs


def weight_stream(step_ms, E):
    """The rollout kernel's weight traffic from L2: every workgroup (16 samples, one per CU at E =
    4096) reads each GEMM weight once per step (fp32 fragments or the split copies' two fp16 planes:
    4 B per weight either way), so per step the chip reads (E / 16) x the parameter bytes from L2."""
    from uavhip._lib import LIB
    n = int(LIB.uavhip_policy_layout(None, 0))
    wg = (E + 15) // 16
    gbs = 4.0 * n * wg / (step_ms * 1e-3) / 1e9
    return {"bytes_per_workgroup_step": 4 * n, "workgroups": wg, "achieved": gbs, "peak": L2_PEAK_GBS,
            "unit": "GB/s (L2 -> CU, chip-wide)", "frac": gbs / L2_PEAK_GBS,
            "per_cu_gbs": gbs / min(wg, 256)}


def check_traffic(traffic, ms):
    """Consistency of a PMC byte count with a measured time: bytes / time must not exceed the HBM peak
    (a traffic figure from another code state, or a time that is not the traffic's, would). Returns
    (traffic or None if dropped, implied GB/s, within peak, reason)."""
    if traffic is None or ms is None:
        return traffic, None, None, None
    gbs = traffic / (ms * 1e-3) / 1e9
    if gbs <= HBM_PEAK_GBS:
        return traffic, gbs, True, None
    return None, gbs, False, (f"traffic {traffic / 1e6:.1f} MB per step over {ms * 1e3:.2f} us implies "
                              f"{gbs:.0f} GB/s > HBM peak: traffic dropped")


def env_bytes_per_step(M):
    return 24 * M + 490


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--uavs", type=int, default=16)
    ap.add_argument("--targets", type=int, default=32)
    ap.add_argument("--horizon", type=int, default=64)
    ap.add_argument("--ppo-minibatch", type=int, default=4096)
    ap.add_argument("--no-ppo", action="store_true")
    ap.add_argument("--no-env-fused", action="store_true", help="skip the env-only fused multi-step lines")
    ap.add_argument("--ppo-impl", choices=["fused", "torch-graph", "torch-eager"], default="fused",
                    help="PPO update implementation timed for ppo_samples_per_s")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end rollout + update iteration legs")
    ap.add_argument("--no-env-diff", action="store_true",
                    help="skip the env step's live differential and phase share (child processes; A/B runs)")
    ap.add_argument("--rccl-gather", action="store_true",
                    help="N > 1: only the collective all-gather after each rollout (no pipelined peer-to-peer "
                         "copies, uavhip.dist.IpcAllGather); by default the faster of the two, measured, is timed")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the dropin_loop leg (main_train.py's loop at E = 1 through the drop-ins)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--ppo-timeout", type=float, default=300.0,
                    help="N > 1: the data-parallel update leg's watchdog (s); on expiry the line prints without it")
    ap.add_argument("--eager", action="store_true", help="launch kernels eagerly instead of replaying a hipGraph")
    ap.add_argument("--unfused", action="store_true",
                    help="separate policy and env launches per step instead of uavhip_rollout_step")
    ap.add_argument("--per-step-launch", action="store_true",
                    help="one fused launch per rollout step instead of one launch per iteration")
    ap.add_argument("--full-window", action="store_true",
                    help="policy forward over the full window every step (no window-row ring)")
    return ap.parse_args()


def cpu_baseline(args, state_dict, seconds):
    """The CPU port on the host cores: C oracle env.step + torch fp32 policy (oracle.policy_ref)."""
    import random
    import oracle
    from oracle import gae as ogae
    from oracle import policy_ref
    from uavhip.config import Config, params_vector
    from uavhip.scene import generate_scene
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    torch.set_num_threads(cores)
    c = Config()
    c.NUM_UAVS, c.NUM_TARGETS = args.uavs, args.targets
    np.random.seed(0); random.seed(0)
    E = 64
    prm = params_vector(c)
    envs = [oracle.OracleEnv(generate_scene(c), prm) for _ in range(E)]
    obs = np.stack([e.reset() for e in envs])
    sd = {k: v.detach().float().cpu() for k, v in state_dict.items()}
    rng = np.random.default_rng(0)
    steps = 0
    rew_buf, done_buf, val_buf = [], [], []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        with torch.no_grad():
            logits, value = policy_ref.heads(sd, torch.from_numpy(obs))
            p1 = torch.softmax(logits, -1)[:, 1].numpy()
        acts = (rng.random(E) < p1).astype(np.int64)
        rw = np.zeros(E); dn = np.zeros(E, np.uint8)
        for i, e in enumerate(envs):
            o, r, d, _ = e.step(int(acts[i]))
            rw[i], dn[i] = r, d
            obs[i] = e.reset() if d else o
        rew_buf.append(rw); done_buf.append(dn); val_buf.append(value.numpy())
        steps += E
        if len(rew_buf) == 64:
            ogae.gae_2d(np.stack(rew_buf), np.stack(done_buf), np.stack(val_buf))
            rew_buf, done_buf, val_buf = [], [], []
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{E} envs x {steps // E} steps of {args.uavs}x{args.targets} ({dt:.1f} s): torch-CPU fp32 "
                      f"policy forward ({cores} threads) + C oracle UAVEnv.step (1 thread) + numpy GAE"}


def cpu_env_baseline(args, seconds=10.0):
    """UAVEnv.step alone on the host cores (north_star: the reference CPU env.step timed on the same
    box): the C oracle's batched loop in one process per core, run as a child process that never
    touches the GPU (oracle/cpu_env_bench.py)."""
    import subprocess
    procs = max(1, min(16, len(os.sched_getaffinity(0))))
    out = subprocess.run([sys.executable, "-m", "oracle.cpu_env_bench", "--procs", str(procs), "--seconds",
                          str(seconds), "--uavs", str(args.uavs), "--targets", str(args.targets)],
                         cwd=ROOT, capture_output=True, text=True, timeout=seconds + 120, check=True)
    return json.loads(out.stdout.strip().splitlines()[-1])


def env_fused_rate(E, N, M, T, dev, reps=5, obs_dtype=torch.float32):
    """Env-only multi-step launch (BASELINE configs[1] shape; K2r / K2, see env.hip's dispatch): one
    launch steps E envs T times with state in registers (Bernoulli(0.5) actions drawn on device beforehand, auto-reset, obs / reward / done /
    info written every step). Returns env-steps/s and algorithmic GB/s (SURVEY 8d units; fp16 obs
    write 140 B instead of 280 B per env-step)."""
    from uavhip.vec_env import VecUAVEnv
    env = VecUAVEnv(E, N, M, 1, 1, seed=77, full_reset_period=200, obs_dtype=obs_dtype)
    env.generate_scenes()
    env.reset(episode=1)
    g = torch.Generator(device=dev).manual_seed(5)
    acts = torch.randint(0, 2, (T, E), generator=g, device=dev, dtype=torch.int8)
    obs = torch.empty(T, E, 5, 14, device=dev, dtype=obs_dtype)
    rew = torch.empty(T, E, dtype=torch.float64, device=dev)
    done = torch.empty(T, E, dtype=torch.uint8, device=dev)
    info = torch.empty(T, E, 8, dtype=torch.float64, device=dev)
    for _ in range(2):
        env.step(acts, obs_out=obs, reward_out=rew, done_out=done, info_out=info)
        env.refresh_scenes()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for _ in range(reps):
        e0.record()
        env.step(acts, obs_out=obs, reward_out=rew, done_out=done, info_out=info)
        e1.record()
        env.refresh_scenes()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    t = float(np.median(ms)) * 1e-3
    rate = E * T / t
    f16 = obs_dtype == torch.float16
    bps = env_bytes_per_step(M) - (140 if f16 else 0)
    gbs = bps * rate / 1e9
    return {"workload": f"{E} envs x {N} UAV x {M} tgt, {T} fused steps per launch" + (", fp16 obs" if f16 else ""),
            "value": rate, "unit": "env-steps/s", "ms_per_launch": t * 1e3, "achieved": gbs, "peak": HBM_PEAK_GBS,
            "unit_roofline": f"GB/s (algorithmic 24*M + {490 - 140 * f16} B per env-step)", "frac": gbs / HBM_PEAK_GBS}


def score_pairs_rate(E, N, M, dev, reps=5):
    """K1 (LDS-tiled pair scoring, one workgroup per env) over E fresh scenes: pairs/s and the
    algorithmic 8 + 48/M + 40/N B per pair + 8 B per UAV against HBM. fp64-VALU bound
    (acos + 2 exp + sqrt + 3 divisions per pair)."""
    from uavhip.vec_env import VecUAVEnv
    env = VecUAVEnv(E, N, M, 1, 1, seed=78, full_reset_period=0)
    env.generate_scenes()
    env.score_pairs()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for _ in range(reps):
        e0.record()
        env.score_pairs()
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    t = float(np.median(ms)) * 1e-3
    pairs = E * N * M
    gbs = (pairs * (8 + 48 / M + 40 / N) + 8 * E * N) / t / 1e9
    return {"workload": f"K1 score_pairs, {E} envs x {N} UAV x {M} tgt", "value": pairs / t, "unit": "pairs/s",
            "ms_per_launch": t * 1e3, "achieved": gbs, "peak": HBM_PEAK_GBS,
            "unit_roofline": "GB/s (algorithmic 8 + 48/M + 40/N B per pair + 8 B per UAV)", "frac": gbs / HBM_PEAK_GBS}


def ppo_update_rate(args, eng, policy, world, dist, dev, E, T):
    """Time one PPO update (5 epochs) over the iteration's trajectories; see the module docstring."""
    from uavhip.ppo import GraphPPOUpdater, make_optimizer, ppo_epochs
    tr = eng.traj
    n = E * T
    states = tr.obs[:T].reshape(n, 5, 14)
    acts = tr.actions.reshape(n).long()
    bufs = (states, acts, tr.logp.reshape(n), tr.values.reshape(n), tr.ret.reshape(n), tr.adv.reshape(n))
    if world > 1:  # the update runs on the all-gathered batch, data parallel over the ranks
        g = eng.gather()  # this iteration's gathered batch (cached by the timed loop's call)
        bufs = (g["obs"], g["actions"], g["logp"], g["values"], g["returns"], g["advantages"])
        n = bufs[0].shape[0]
    if args.ppo_impl == "torch-eager":
        opt = make_optimizer(policy)
        impl = "torch autograd on GPU, eager launches"
        run = lambda: ppo_epochs(policy, opt, *bufs, batch_size=args.ppo_minibatch)  # noqa: E731
    elif args.ppo_impl == "torch-graph":
        opt = make_optimizer(policy, capturable=True)
        upd = GraphPPOUpdater(policy, opt, *bufs, args.ppo_minibatch)
        upd.capture()  # once per buffer set (not timed): replays cover every later update
        impl = "torch autograd on GPU, minibatch step captured in a hipGraph"
        run = upd.run
    else:
        from uavhip.train import FusedPPOTrainer
        # global minibatch = per-GPU minibatch x world (each rank runs its slice of every step)
        trainer = FusedPPOTrainer(policy, args.ppo_minibatch * world)
        trainer.set_buffers(*bufs)
        if world == 1:
            trainer.capture()  # once per buffer set (not timed): replays cover every later update
            impl = ("HIP training step (uavhip_ppo_step: fused forward / backward kernels, weight-gradient "
                    "MFMA GEMM (chunked, XCD-aware), fused clip + Adam), one hipGraph replay per epoch")
        else:
            impl = ("HIP training step, data parallel: forward / all-reduce loss sums / backward / "
                    "all-reduce grads / clip+Adam per global minibatch")
            graphed = False
            if trainer.graph_collectives:  # RCCL: the epoch with its all-reduces as one graph (not timed)
                # collective: the ranks vote inside capture(); None on every rank if any rank failed
                graphed = trainer.capture() is not None
            if graphed:
                impl += ", one hipGraph replay per epoch with the RCCL all-reduces captured"
            else:
                impl += f", eager ({dist.get_backend()} collectives)"
        gen = torch.Generator().manual_seed(1234)  # same minibatch order on every rank
        use_graph = world == 1 or bool(trainer.graphs)
        run = lambda: trainer.run(generator=gen, use_graph=use_graph)  # noqa: E731
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    p0 = time.perf_counter()
    _, _, _, cnt = run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    pdt = time.perf_counter() - p0
    if dist is not None:
        t = torch.tensor([pdt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        pdt = t.item()
    se = n * 5 / pdt
    # whole-node MFMA rate of the update: SURVEY 8(d)'s algorithmic training work (3 x the dense
    # forward per sample-epoch) and the work the HIP step executes (last layers pruned: forward 2.45
    # + input gradients 2.62 + weight gradients 2.39 MFLOP), over all GPUs
    alg_tf = se * TRAIN_FLOP_PER_SAMPLE_EPOCH / 1e12
    exe_tf = se * TRAIN_EXEC_FLOP_PER_SAMPLE_EPOCH / 1e12
    # the MFMA peak of the executed FLOP mix (per GPU, x world): split products at 16/3 (forward, dX)
    # and 16/6 (weight gradients) x the f32 MFMA rate, the rest on the f32 MFMA
    split2 = TRAIN_FWD_SPLIT_FLOP + TRAIN_DX_SPLIT_FLOP
    f32_flop = TRAIN_EXEC_FLOP_PER_SAMPLE_EPOCH - split2 - TRAIN_WGRAD_FLOP
    mix_s = (split2 / MFMA_SPLIT_PEAK_TFLOPS + TRAIN_WGRAD_FLOP / MFMA_SPLIT3_PEAK_TFLOPS
             + f32_flop / MFMA_F32_PEAK_TFLOPS)
    peak = TRAIN_EXEC_FLOP_PER_SAMPLE_EPOCH / mix_s * world
    return {"value": n / pdt, "unit": "PPO samples/s (whole node: transitions in the update batch / update "
           "wall time, 5 epochs)", "epochs": 5, "minibatch_per_gpu": args.ppo_minibatch,
           "global_minibatch": args.ppo_minibatch * world, "optimizer_steps": cnt, "batch": n,
           "sample_epochs_per_s": se, "impl": impl,
           "roofline": {"bound": "mfma", "unit": "TFLOP/s (fp32-accurate)", "peak": peak, "achieved": exe_tf,
                        "frac": exe_tf / peak,
                        "peak_source": "MFMA peak of the executed FLOP mix (forward GEMMs and the encoder input "
                                       "gradients as two-plane split products, weight gradients as three-plane, "
                                       "embeddings and heads on the f32 MFMA)",
                        # round 2's measure (every FLOP priced on the f32 MFMA, 157.3 TFLOP/s per GPU)
                        "f32_mfma_equivalent_frac": exe_tf / (MFMA_F32_PEAK_TFLOPS * world),
                        "algorithmic_achieved": alg_tf,
                        "flop_per_sample_epoch": TRAIN_FLOP_PER_SAMPLE_EPOCH,
                        "flop_source": "SURVEY.md 8(d): 3 x the dense forward (4.04 MFLOP) per sample-epoch",
                        "executed_flop_per_sample_epoch": TRAIN_EXEC_FLOP_PER_SAMPLE_EPOCH,
                        "executed_achieved": exe_tf, "executed_frac": exe_tf / peak,
                        "timing": "update wall time (all kernels of the step, launches included)"}}


def ppo_mb64_rate(policy, eng, E, T, dev, n_sub=16384):
    """The reference's own minibatch (BATCH_SIZE = 64, ppo.py:110-115) on the HIP training step: one
    5-epoch update over the first n_sub transitions of the iteration's batch = 5 n_sub / 64 Adam
    steps, each epoch one captured hipGraph of n_sub / 64 minibatch steps (capture not timed), on a
    copy of the policy. Parity mode: the same optimizer trajectory as the reference's update."""
    from uavhip.policy import TransformerActorCritic
    from uavhip.train import FusedPPOTrainer
    tr_ = eng.traj
    n = E * T
    bufs = (tr_.obs[:T].reshape(n, 5, 14), tr_.actions.reshape(n), tr_.logp.reshape(n), tr_.values.reshape(n),
            tr_.ret.reshape(n), tr_.adv.reshape(n))
    n_sub = min(n_sub, n)
    pol = TransformerActorCritic().to(dev)
    pol.load_state_dict(policy.state_dict())
    trainer = FusedPPOTrainer(pol, 64)
    trainer.stage(*(b[:n_sub] for b in bufs))
    trainer.capture()
    gen = torch.Generator().manual_seed(4321)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, _, _, cnt = trainer.run(generator=gen)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"value": n_sub / dt, "unit": "PPO samples/s (transitions / update wall time, 5 epochs)",
            "minibatch": 64, "batch": n_sub, "optimizer_steps": cnt, "ms_per_optimizer_step": dt / cnt * 1e3,
            "impl": "HIP training step at the reference's minibatch 64, one hipGraph replay per epoch"}


def e2e_iteration_rate(eng, policy, E, T, minibatch, iters=2):
    """The loop the reference runs (main_train.py:109-146): a rollout iteration, then the PPO update
    (5 epochs) over ALL of its E * T transitions at `minibatch`, then the next rollout on the updated
    weights -- timed end to end on the host clock (device-synchronised at both ends), with the phase
    split from HIP events on the launch stream. One process, N = 1. The trainer's buffers are views
    of the engine's trajectory (every rollout writes them in place); the update's epoch graph (or its
    256-step chunk graph, FusedPPOTrainer.max_graph_steps) is captured once before the timed loop.
    Returns env-steps/s including the update and the per-phase times."""
    from uavhip.train import FusedPPOTrainer
    tr = eng.traj
    n = E * T
    trainer = FusedPPOTrainer(policy, minibatch)
    trainer.set_buffers(tr.obs[:T].reshape(n, 5, 14), tr.actions.reshape(n), tr.logp.reshape(n),
                        tr.values.reshape(n), tr.ret.reshape(n), tr.adv.reshape(n))
    gen = torch.Generator().manual_seed(99)
    eng.collect()
    trainer.capture()  # not timed (once per buffer set)
    trainer.run(generator=gen)  # warm-up iteration's update
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = 0
    for i in range(iters):
        ev[i][0].record()
        eng.collect()  # graph replay; repacks the policy's inference weights after the update
        ev[i][1].record()
        steps += trainer.run(generator=gen)[3]
        ev[i][2].record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    roll = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    upd = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))
    return {"value": n * iters / dt, "unit": "env-steps/s including the PPO update (rollout + GAE + 5-epoch update "
            "over every transition, serial, as main_train.py runs them)", "minibatch": minibatch,
            "iterations": iters, "ms_per_iteration": dt / iters * 1e3, "rollout_ms": roll, "update_ms": upd,
            "update_share": upd / (roll + upd), "optimizer_steps_per_iteration": steps // iters,
            "ms_per_optimizer_step": upd / max(1, steps // iters),
            "ppo_samples_per_s": n / (upd * 1e-3),
            "timing": "host clock over the loop; phase split from HIP events around the rollout replay and the update"}


def dropin_loop_rate(N, M, seconds, cpu_seconds=None):
    """The reference's own training loop (main_train.py:79-146) at E = 1 through the drop-ins
    (envs.uav_env.UAVEnv over the HIP env kernel, agents.ppo.PPOAgent over the fused forward and the
    HIP training step at the reference's minibatch 64): per episode reset + the first state's value,
    per step select_action -> step -> store_transition, update() when the buffer holds >= 4 x 64
    transitions. Warm-up up to and including the third update (captures the epoch graphs of the
    common buffer lengths), then timed for `seconds`. Host syncs per env step: select_action's one
    device->host copy of (action, finite flag) and step's one 368-byte copy of the step's outputs.
    Beside it, the CPU port of the same loop (oracle/cpu_loop_bench.py: C oracle env + torch-CPU
    forward + torch-CPU autograd update, 1 thread) in a child process."""
    import random
    import subprocess
    from agents.ppo import PPOAgent
    from envs.uav_env import UAVEnv
    from uavhip.config import cfg
    saved = (cfg.NUM_UAVS, cfg.NUM_TARGETS)
    cfg.NUM_UAVS, cfg.NUM_TARGETS = N, M
    try:
        np.random.seed(0)
        random.seed(0)
        torch.manual_seed(0)
        env, agent = UAVEnv(), PPOAgent()
        st = dict(steps=0, roll_s=0.0, upd_s=0.0, upd_samples=0, updates=0, episodes=0)

        def episode(i):
            state = env.reset(full_reset=(i == 1 or i % 200 == 0))
            with torch.no_grad():  # main_train.py:87-93
                agent.policy_old.get_action(torch.as_tensor(state).unsqueeze(0).to(agent.device))[2].item()
            done, n = False, 0
            while not done:
                a = agent.select_action(state)
                state, r, done, _ = env.step(a)
                agent.store_transition(r, done)
                n += 1
            return n

        i = warm_updates = 0
        while warm_updates < 3:
            i += 1
            episode(i)
            if len(agent.buffer["states"]) >= cfg.BATCH_SIZE * 4:
                agent.update()
                warm_updates += 1
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        while time.perf_counter() - t_start < seconds:
            i += 1
            t0 = time.perf_counter()
            st["steps"] += episode(i)
            st["roll_s"] += time.perf_counter() - t0
            st["episodes"] += 1
            if len(agent.buffer["states"]) >= cfg.BATCH_SIZE * 4:
                nb = len(agent.buffer["states"])
                t1 = time.perf_counter()
                agent.update()
                torch.cuda.synchronize()
                st["upd_s"] += time.perf_counter() - t1
                st["upd_samples"] += nb
                st["updates"] += 1
        total = time.perf_counter() - t_start
    finally:
        cfg.NUM_UAVS, cfg.NUM_TARGETS = saved
    res = {"workload": f"E = 1, {N} UAV x {M} tgt: main_train.py:79-146 through envs.uav_env.UAVEnv / agents.ppo.PPOAgent",
           "value": st["steps"] / total, "unit": "env-steps/s (loop wall time, updates included)",
           "rollout_env_steps_per_s": st["steps"] / st["roll_s"],
           "update_samples_per_s": st["upd_samples"] / st["upd_s"] if st["upd_s"] > 0 else None,
           "update_unit": "transitions per update() wall time (5 epochs at minibatch 64, HIP training step)",
           "host_syncs_per_env_step": 2,
           "host_syncs": "select_action: one device->host copy of (action, finite flag); UAVEnv.step: one 368-byte "
                         "copy of obs / reward / info / done; plus one per episode (the first state's value)",
           "episodes": st["episodes"], "updates": st["updates"], "seconds": total}
    try:
        out = subprocess.run([sys.executable, "-m", "oracle.cpu_loop_bench", "--uavs", str(N), "--targets", str(M),
                              "--seconds", str(cpu_seconds or seconds), "--threads", "1"],
                             cwd=ROOT, capture_output=True, text=True, timeout=(cpu_seconds or seconds) + 180, check=True)
        res["cpu_baseline"] = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception as exc:  # the headline line must still print
        res["cpu_baseline"] = {"value": None, "error": repr(exc)}
    return res


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus, environ, device_count=None):
    """How `bench.py --gpus N` runs. Returns one of
      ("run", world)       -- this process is a rank (WORLD_SIZE set by a launcher, or N = 1);
      ("spawn", [env, ...]) -- N > 1 and no launcher: start N rank processes with these environments
                              (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
                              MASTER_PORT), relay rank 0's line, exit with the worst rank's code;
      ("error", message)   -- WORLD_SIZE disagrees with --gpus, N < 1, or more RCCL ranks than devices
                              (RCCL runs one rank per device; BENCH_DIST_BACKEND=gloo rehearses N ranks
                              on fewer GPUs).
    Decided before anything touches the GPU (device_count: torch.cuda.device_count(), which does not
    initialise the device on this image)."""
    if gpus < 1:
        return ("error", f"--gpus {gpus}: need at least one GPU")
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            return ("error", f"WORLD_SIZE={ws} from the launcher but --gpus {gpus}: they must agree")
        return ("run", int(ws))
    if gpus == 1:
        return ("run", 1)
    backend = environ.get("BENCH_DIST_BACKEND", "nccl")
    if backend == "nccl" and device_count is not None and device_count < gpus:
        return ("error", f"--gpus {gpus} over RCCL needs {gpus} devices, {device_count} visible "
                         f"(BENCH_DIST_BACKEND=gloo rehearses the ranks on fewer GPUs)")
    port = str(_free_port())
    envs = []
    for r in range(gpus):
        e = dict(environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC: the only mode the host driver supports
        envs.append(e)
    return ("spawn", envs)


def spawn_ranks(envs, argv, grace_s=120.0, script=None):
    """Run one bench.py process per rank (child processes; this parent never touches the GPU).
    The children share this process's stdout / stderr, so rank 0's JSON line is the parent's output.
    If a rank fails, the others get `grace_s` to finish (they may wait in a collective for it), then
    are terminated. Returns the worst exit code (0 only if every rank exited 0)."""
    import signal
    import subprocess
    script = script or os.path.abspath(__file__)
    procs = [subprocess.Popen([sys.executable, script] + list(argv), env=e) for e in envs]

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        failed_at = None
        while any(p.poll() is None for p in procs):
            if failed_at is None and any(p.returncode not in (None, 0) for p in procs):
                failed_at = time.monotonic()
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                time.sleep(10)
                for p in procs:
                    if p.poll() is None:
                        p.kill()
            time.sleep(0.2)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    if bad:
        print(f"[bench] rank exit codes {codes}", file=sys.stderr)
        return bad[0] if bad[0] > 0 else 1
    return 0


def run_with_watchdog(fn, timeout_s, on_timeout):
    """fn() with a watchdog thread: if it has not returned after timeout_s, on_timeout() runs (rank 0
    prints the line) and the process exits 0 at once (os._exit: a rank blocked in a collective never
    returns to let a normal exit run). Used for the N > 1 data-parallel update leg, whose collectives
    could otherwise hold back every rank's exit and the rollout line with them."""
    import threading

    def fire():
        try:
            on_timeout()
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)
    t = threading.Timer(timeout_s, fire)
    t.daemon = True
    t.start()
    try:
        return fn()
    finally:
        t.cancel()


def main():
    args = parse()
    plan = launch_plan(args.gpus, os.environ, device_count=torch.cuda.device_count())
    if plan[0] == "error":
        print(f"[bench] {plan[1]}", file=sys.stderr)
        sys.exit(2)
    if plan[0] == "spawn":
        sys.exit(spawn_ranks(plan[1], sys.argv[1:]))
    world = plan[1]
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # BENCH_DIST_BACKEND=gloo rehearses the N > 1 code path with several ranks on one GPU
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from uavhip.policy import TransformerActorCritic
    from uavhip.rollout import RolloutEngine
    from uavhip.vec_env import VecUAVEnv

    E, T = args.envs, args.horizon
    torch.manual_seed(0)  # identical initial policy on every rank
    policy = TransformerActorCritic().to(dev)
    # rank r owns envs [r E, (r + 1) E) of the node's world * E: its scenes and action samples are
    # those of the same envs in a one-process run over all of them (env_base / total_envs)
    env = VecUAVEnv(E, args.uavs, args.targets, 1, 1, seed=1, full_reset_period=200, env_base=rank * E)
    eng = RolloutEngine(env, policy, T, want_info=True, bootstrap=True, seed=1000, normalize=(world == 1),
                        row_cache=not args.full_window, fused_step=False if args.unfused else None,
                        total_envs=world * E, persistent=False if args.per_step_launch else None)
    eng.start()

    # The iteration is captured once into a hipGraph and replayed. HIP events (recorded on the
    # launch stream around every policy / env launch) cannot live inside a ROCm graph, so the LAST
    # timed iteration runs the same body as eager launches and carries the events: the kernel
    # timings are live, from inside the timed region.
    use_graph = not args.eager
    mode = "hipGraph replay (last iteration eager, with HIP events)" if use_graph else "eager launches"
    eng.enable_events(external=False)
    if use_graph:
        try:
            eng.capture()
        except Exception as exc:  # graph capture unavailable: measure eager launches instead
            print(f"[bench] graph capture failed ({exc!r}); falling back to eager launches", file=sys.stderr)
            eng.graph = None
            mode = "eager launches (graph capture failed)"

    # N > 1: the exchange pipelined one iteration behind the rollout (peer-to-peer copies out of
    # IPC-mapped buffers on a side stream, beside the next rollout; host sync over a gloo group), or
    # one RCCL all-gather after each rollout (--rccl-gather, or when the IPC mapping fails on any rank)
    xchg, xchg_err = None, None
    if dist is not None and not args.rccl_gather:
        from uavhip.dist import IpcAllGather, compact_floats
        host_group = dist.new_group(backend="gloo")
        try:
            xchg = IpcAllGather(compact_floats(T, E), dev, host_group)
        except Exception as exc:
            xchg_err = repr(exc)
        ok = torch.tensor([0 if xchg is None else 1], device=dev, dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not ok.item():
            xchg = None
            xchg_err = xchg_err or "the IPC mapping failed on another rank"

    def it_gather(eager=False):  # the exchange as one collective all-gather after the rollout
        eng.collect(eager=eager)
        if dist is not None:
            eng.gather()

    def it_pipelined(eager=False):  # the exchange as peer copies beside the next rollout
        eng.collect(eager=eager)
        if xchg.pending is not None:
            eng.gather_finish(xchg)  # the previous iteration's exchange, beside this rollout
        eng.gather_submit(xchg)

    def drain():
        if xchg is not None and xchg.pending is not None:
            eng.gather_finish(xchg)
            eng.gather()

    def pipelined_check():
        """The last drained pipelined exchange (the engine's current iteration) against the collective
        all_gather of the same payloads, bitwise, on every rank."""
        from uavhip.dist import all_gather_rows, pack_compact
        tr_ = eng.traj
        ref = all_gather_rows(pack_compact(tr_.obs, tr_.actions, tr_.logp, tr_.values, tr_.ret, tr_.adv,
                                           tr_.dones).view(1, -1))
        same = torch.tensor([int(torch.equal(ref, xchg.recv[(xchg.k - 1) & 1]))], device=dev, dtype=torch.int32)
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
        return bool(same.item())

    def per_iteration_ms(body, n):  # steady state, untimed region: max over ranks
        torch.cuda.synchronize()
        dist.barrier()
        a = time.perf_counter()
        for _ in range(n):
            body()
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([(time.perf_counter() - a) / n * 1e3], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item()

    for _ in range(args.warmup):
        it_gather()
    iteration, calibration = it_gather, None
    if dist is not None:
        # N > 1: the exchange the timed loop uses is chosen by measurement: a few
        # untimed steady-state iterations of each, max over ranks; the faster one runs the timed loop
        calibration = {"iterations_each": 3, "collective_ms_per_iteration": per_iteration_ms(it_gather, 3),
                       "collective": f"{dist.get_backend()} all-gather after each rollout"}
        if xchg is not None:
            it_pipelined()  # fills the pipeline: every timed call below finishes one exchange and submits one
            calibration["pipelined_ms_per_iteration"] = per_iteration_ms(it_pipelined, 3)
            drain()
            calibration["pipelined_check"] = pipelined_check()
            if calibration["pipelined_ms_per_iteration"] < calibration["collective_ms_per_iteration"]:
                iteration = it_pipelined
        calibration["chosen"] = "pipelined" if iteration is it_pipelined else "collective"
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        iteration(eager=(i == args.steps - 1))
    drain()  # the last iteration's pipelined exchange (exposed: inside the timed region)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    env_steps = E * T * args.steps * world
    value = env_steps / elapsed

    exchange = None
    if dist is not None:  # the exchange used, how it was chosen, and the pipelined copies checked
        pipelined = iteration is it_pipelined
        exchange = {"kind": "peer-to-peer copies out of IPC-mapped buffers, pipelined beside the next rollout"
                    if pipelined else f"{dist.get_backend()} all-gather after each rollout",
                    "fallback_reason": xchg_err, "calibration": calibration,
                    "check": pipelined_check() if pipelined else calibration.get("pipelined_check"),
                    "check_what": ("the gathered payloads of the last " + ("timed" if pipelined else "calibration")
                                   + " iteration's pipelined exchange == the collective all_gather of the same "
                                   "payloads, bitwise, every rank") if xchg is not None else None}

    timeline = None
    if dist is not None:  # one more iteration, untimed, with the phases separated: rollout | exchange
        torch.cuda.synchronize()
        dist.barrier()
        a = time.perf_counter()
        eng.collect()
        torch.cuda.synchronize()
        b = time.perf_counter()
        if xchg is not None:
            eng.gather_submit(xchg)
            eng.gather_finish(xchg)
        eng.gather()
        torch.cuda.synchronize()
        c = time.perf_counter()
        t = torch.tensor([b - a, c - b], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        timeline = {"rollout_ms": t[0].item() * 1e3, "exchange_ms": t[1].item() * 1e3,
                    "exchange": "global advantage moments all-reduce + compact trajectory all-gather + window rebuild",
                    "backend": dist.get_backend(),
                    "timing": "one extra iteration after the timed region, host clock with a device sync between "
                              "the phases, max over ranks"}

    # the last timed iteration's launches: T+1 policy and T env launches, or (fused steps) T fused
    # forward + env-step launches and the bootstrap forward (the same kernel without the env step)
    pol_list, env_list = eng.event_ms()
    env_phase = env_err = env_diff = None
    if eng.fused_step:
        pol_ms = float(np.mean(pol_list[:T]))
        env_ms = None
        if eng.persistent and rank == 0 and world == 1 and not args.no_env_diff:
            # the env step's cost = the compiled-out differential (product minus NOENV build, HIP
            # events, child processes on this box); the TRACE build's phase share is a diagnostic
            env_diff, env_err = env_differential(args)
            if env_diff is not None and env_diff["env_ms"] > 0:
                # the differential's share of its own product time, applied to the headline kernel's
                # time (the child runs replay the iteration warm like the bench; the share carries the
                # measurement to the headline's operating point either way)
                env_diff["share"] = env_diff["env_ms"] / env_diff["product_ms"]
                env_diff["product_vs_headline"] = env_diff["product_ms"] / pol_ms
                env_ms = env_diff["share"] * pol_ms
            elif env_diff is not None:
                env_err = f"non-positive differential {env_diff['env_ms']:.4f} ms"
            env_phase, phase_err = env_phase_share(args)
            if phase_err:
                env_err = (env_err + "; " if env_err else "") + "phase share: " + phase_err
        elif not eng.persistent:  # per-step launches: the fused launch minus the bootstrap forward
            env_ms = max(float(np.mean(pol_list[:T])) - float(pol_list[T]), 1e-6)
    else:
        pol_ms = float(np.mean(pol_list))
        env_ms = float(np.mean(env_list))
    flop_exec = ROWS_FLOP_PER_SAMPLE if eng.rowproj is not None else POLICY_FLOP_PER_SAMPLE
    achieved_tf = POLICY_FLOP_PER_SAMPLE * E / (pol_ms * 1e-3) / 1e12
    exec_tf = flop_exec * E / (pol_ms * 1e-3) / 1e12
    # the MFMA peak of the FLOP mix: split products at 16/3 x the f32 rate, the rest on the f32 MFMA.
    # The algorithmic count prices the ring's skipped layer-0 rows as the same split products.
    split = SPLIT_FLOP_PER_SAMPLE_ROWS if eng.rowproj is not None else SPLIT_FLOP_PER_SAMPLE
    mix_peak = lambda flop, sp: flop / ((flop - sp) / MFMA_F32_PEAK_TFLOPS  # noqa: E731
                                        + sp / MFMA_SPLIT_PEAK_TFLOPS)
    split_alg = split + (POLICY_FLOP_PER_SAMPLE - flop_exec)
    peak_alg, peak_exec = mix_peak(POLICY_FLOP_PER_SAMPLE, split_alg), mix_peak(flop_exec, split)
    env_gbs = None if env_ms is None else env_bytes_per_step(args.targets) * E / (env_ms * 1e-3) / 1e9

    env_fused = stress = None
    if rank == 0 and world == 1 and not args.no_env_fused:
        env_fused = [env_fused_rate(1024, 8, 16, 256, dev), env_fused_rate(E, args.uavs, args.targets, 256, dev),
                     env_fused_rate(8192, 64, 128, 64, dev, obs_dtype=torch.float16)]
        # the kernel uavhip_env_step dispatches for each leg (env.hip): K2r wherever omega = 0 and
        # M <= 32 (512-thread workgroups of 4 envs: 128 threads per env), K2 one env per wave (M > 32,
        # 256-thread workgroups of 4 envs); matched to the profile by name and launch grid
        for leg, (kern, grid) in zip(env_fused, (("k_env_replay", 128 * 1024), ("k_env_replay", 128 * E),
                                                 ("k_env_step", 64 * 8192))):
            leg["counters"] = env_counters(kern, grid)
            leg["kernel"] = leg["counters"]["kernel"] if leg["counters"] else kern
        stress = score_pairs_rate(8192, 64, 128, dev)
        stress["counters"] = env_counters("k_score_pairs", 256 * 8192)

    ppo = ppo64 = None
    if not args.no_ppo and world == 1 and args.ppo_impl == "fused":
        try:
            ppo64 = ppo_mb64_rate(policy, eng, E, T, dev)
        except Exception as exc:  # the headline rollout line must still print
            print(f"[bench] minibatch-64 PPO measurement failed: {exc!r}", file=sys.stderr)
            ppo64 = {"value": None, "error": repr(exc)}
    def ppo_leg():
        try:
            return ppo_update_rate(args, eng, policy, world, dist, dev, E, T)
        except Exception as exc:  # the headline rollout line must still print
            print(f"[bench] PPO update measurement failed: {exc!r}", file=sys.stderr)
            return {"value": None, "error": repr(exc)}
    if not args.no_ppo and world == 1:
        ppo = ppo_leg()

    e2e = None
    if not args.no_ppo and not args.no_e2e and world == 1 and args.ppo_impl == "fused":
        e2e = {}
        for mb, it in ((args.ppo_minibatch, 3), (64, 1)):
            try:
                e2e[f"minibatch_{mb}"] = e2e_iteration_rate(eng, policy, E, T, mb, iters=it)
            except Exception as exc:  # the headline rollout line must still print
                print(f"[bench] end-to-end iteration at minibatch {mb} failed: {exc!r}", file=sys.stderr)
                e2e[f"minibatch_{mb}"] = {"value": None, "error": repr(exc)}

    dropin = None
    if rank == 0 and world == 1 and not args.no_dropin:
        dropin = []
        for N_, M_ in ((30, 10), (args.uavs, args.targets)):
            try:
                dropin.append(dropin_loop_rate(N_, M_, 6.0))
            except Exception as exc:  # the headline line must still print
                print(f"[bench] dropin loop {N_}x{M_} failed: {exc!r}", file=sys.stderr)
                dropin.append({"workload": f"E = 1, {N_} UAV x {M_} tgt", "value": None, "error": repr(exc)})

    cpu = cpu_env = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, policy.state_dict(), args.cpu_seconds)
        try:
            cpu_env = cpu_env_baseline(args)
        except Exception as exc:  # the headline line must still print
            cpu_env = {"value": None, "error": repr(exc)}

    pol_kernel = ("k_rollout_steps" if eng.persistent else "k_policy_forward<false, true, true>" if eng.fused_step
                  else "k_policy_forward<false, true, false>" if eng.rowproj is not None
                  else "k_policy_forward<false, false, false>")
    pol_traffic, pol_src = profiled_traffic(pol_kernel)
    if pol_traffic is not None and eng.persistent:  # one launch = T steps: per-step bytes
        pol_traffic /= T
    prof_kernel = None
    pk = profiled_kernel_time(pol_kernel)
    if pk is not None:  # rocprofv3 of the same code, same lease as a bench run (scripts/profile.sh)
        per = T if eng.persistent else 1
        prof_kernel = {"kernel": pk["kernel"], "source": pk["source"],
                       "avg_ms_per_step": pk["avg_ns"] * 1e-6 / per,
                       "timed_avg_ms_per_step": pk["timed_avg_ns"] * 1e-6 / per if "timed_avg_ns" in pk else None,
                       "timed_min_ms_per_step": pk["timed_min_ns"] * 1e-6 / per if "timed_min_ns" in pk else None,
                       "launches": pk.get("calls"),
                       "what": "rocprofv3 --kernel-trace --stats of bench.py --steps 10 --warmup 2: average over all "
                               "launches and over the 10 timed ones, per step"}
    env_prof_ns = None
    if eng.persistent:
        env_traffic, env_traffic_src, env_prof_ns = env_share_traffic()
    elif eng.fused_step:
        env_traffic, env_traffic_src = None, None
    else:
        env_traffic, env_traffic_src = profiled_traffic("k_env_step<1, false>")
    env_traffic, env_traffic_gbs, env_traffic_check, why = check_traffic(env_traffic, env_ms)
    if why:
        env_err = (env_err + "; " if env_err else "") + why
    line = None
    if rank == 0:
        line = {
            "metric": "env-steps/sec (whole node), full PPO rollout, 4096 envs x 16 UAV x 32 tgt per GPU",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32 policy (f32 MFMA + fp32-accurate split products on the f16 MFMA) + f64 env",
            "data": "synthetic (on-device Philox scenes, "
            "random-init policy, actions sampled from the policy)",
            "config": {"workload": "BASELINE configs[2]: full rollout (policy fwd -> sample -> env.step) + GAE"
                       + (" + trajectory all-gather (" + ("pipelined peer copies" if iteration is it_pipelined
                                                                     else dist.get_backend() + " all-gather")
                          + ")" if world > 1 else ""),
                       "envs_per_gpu": E, "uavs": args.uavs, "targets": args.targets, "horizon": T,
                       "env_steps_per_step": E * T * world, "parallelism": f"env-sharded x{world}",
                       "full_reset_period": 200, "launch": mode},
            "roofline": {"kernel": pol_kernel, "bound": "mfma", "achieved": achieved_tf,
                         "peak": peak_alg, "unit": "TFLOP/s (fp32-accurate)", "frac": achieved_tf / peak_alg,
                         "peak_source": (f"MFMA peak of the FLOP mix: {split_alg:,} of the {POLICY_FLOP_PER_SAMPLE:,} "
                                         f"FLOP/sample as split products on the f16 cores ({MFMA_SPLIT_PEAK_TFLOPS:.1f} TFLOP/s fp32-"
                                         f"equivalent = 2.5 PF f16 / 3), the rest on the f32 MFMA "
                                         f"({MFMA_F32_PEAK_TFLOPS} TFLOP/s); MI355X_MICROARCH.md"),
                         "traffic": pol_traffic,
                         "traffic_unit": "bytes per step (PMC bytes per launch / T)" if eng.persistent else
                         "bytes/launch (PMC)", "traffic_source": pol_src,
                         "avg_launch_ms": pol_ms,
                         "profiled": prof_kernel,
                         "flop_per_launch": POLICY_FLOP_PER_SAMPLE * E,
                         "flop_per_launch_source": "SURVEY.md 8(d): 2,446,208 FLOP/sample x E",
                         "executed_flop_per_launch": flop_exec * E, "executed_achieved": exec_tf,
                         "executed_peak": peak_exec, "executed_frac": exec_tf / peak_exec,
                         # round 2's measure (every executed FLOP priced on the f32 MFMA, 157.3 TFLOP/s)
                         "f32_mfma_equivalent_frac": exec_tf / MFMA_F32_PEAK_TFLOPS,
                         # the other resource every step of the kernel streams: its weights from L2,
                         # once per step in every workgroup (one 16-sample workgroup per CU)
                         "weight_stream": weight_stream(pol_ms, E),
                         "split_flop_per_launch": split * E,
                         "steps_per_launch": T if eng.persistent else 1,
                         "path": ("fused rollout steps (window-row forward + sample + env step), all T steps of the "
                                  "iteration in one launch (per-step figures = launch / T)" if eng.persistent else
                                  "fused rollout step (window-row forward + sample + env step, one launch)"
                                  if eng.fused_step else "window-row ring (layer-0 in_proj of the new row only)"
                                  if eng.rowproj is not None else "full window"),
                         "timing": ("HIP events around the T-step launch of the last timed iteration, divided by T "
                                    "(env step included)" if eng.persistent else
                                    "HIP events around each of the T fused launches of the last timed iteration "
                                    "(env step included)" if eng.fused_step else
                                    "HIP events around each of the T+1 launches of the last timed iteration")},
            "env_roofline": None if env_ms is None else {
                "kernel": "env step inside k_rollout_steps" if eng.persistent else
                "env step inside the fused rollout launch" if eng.fused_step else "k_env_step",
                "timing": ("the compiled-out differential: k_rollout_steps per step on the product build minus "
                           "on the NOENV build (env step compiled out), HIP events on an eager iteration after warm "
                           "graph replays, median of alternating child-process runs on this box "
                           "(scripts/rollout_run.py); its share of the product time x the headline kernel's time"
                           if eng.persistent else
                           "per-step fused launch minus the bootstrap forward launch" if eng.fused_step else
                           "HIP events around each of the T env launches"),
                "differential": env_diff,
                "profiled_differential_ms": None if env_prof_ns is None else env_prof_ns * 1e-6,
                "phase_share_diagnostic": None if env_phase is None else {
                    "share": env_phase["share"], "share_p10_p90": [env_phase["share_p10"], env_phase["share_p90"]],
                    "share_x_step_ms": env_phase["share"] * pol_ms, "phase_cycles": env_phase["phases"],
                    "what": "TRACE build s_memtime stamps: sample -> env.store over the step (diagnostic only: "
                            "it misses the env step's indirect cost on the policy phases)"},
                "bound": "hbm", "achieved": env_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": env_gbs / HBM_PEAK_GBS, "avg_launch_ms": env_ms,
                "traffic": env_traffic, "traffic_unit": "HBM bytes per step of all E envs (PMC: product minus NOENV)",
                "traffic_source": env_traffic_src, "traffic_gbs_at_this_time": env_traffic_gbs,
                "traffic_within_hbm_peak": env_traffic_check,
                "bytes_per_env_step": env_bytes_per_step(args.targets)},
            "env_roofline_error": env_err,
            "env_fused": env_fused,
            "score_pairs": stress,
            "ppo_samples_per_s": ppo,
            "iteration_timeline": timeline,
            "exchange": exchange,
            "ppo_samples_per_s_mb64": ppo64,
            "e2e_iteration": e2e,
            "dropin_loop": dropin,
            "cpu_baseline": cpu,
            "cpu_env_baseline": cpu_env,
        }
        if exchange is not None and exchange.get("check") is False:
            line["invalid"] = ("the pipelined exchange's gathered payloads differ from RCCL's all_gather of the "
                               "same payloads: the multi-GPU throughput is not valid")
    if not args.no_ppo and world > 1:
        # the data-parallel update leg runs last, under a watchdog on every rank: its collectives (an
        # epoch graph with captured RCCL all-reduces) must not be able to hold back the line of the
        # rollout measured above -- if it has not finished in --ppo-timeout s, rank 0 prints the line
        # with the leg marked timed out and every rank exits 0
        def timed_out():
            if line is not None:
                line["ppo_samples_per_s"] = {"value": None, "error": f"data-parallel update leg timed out after "
                                                                     f"{args.ppo_timeout:.0f} s (watchdog)"}
                print(json.dumps(line), flush=True)
        ppo = run_with_watchdog(ppo_leg, args.ppo_timeout, timed_out)
        if line is not None:
            line["ppo_samples_per_s"] = ppo
    if line is not None:
        print(json.dumps(line), flush=True)
    if dist is not None:
        if xchg is not None:  # unmap the peers' send buffers before any rank (an exporter) exits
            torch.cuda.synchronize()
            dist.barrier()
            xchg.close()
        dist.barrier()
        dist.destroy_process_group()
    if exchange is not None and exchange.get("check") is False:
        sys.exit(1)


if __name__ == "__main__":
    main()
