"""Per-launch cost of the rollout's T = 1 env step vs T = 2, 3 (one env per wave, no LDS table),
graph-replayed back to back so launch gaps are excluded: kernel time = fixed + T x per-step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "target-allocation-ppo-transformer_amd"))
import torch  # noqa: E402

from uavhip.vec_env import VecUAVEnv  # noqa: E402

E = int(os.environ.get("E", "4096"))
dev = torch.device("cuda")
for T in (1, 2, 3):
    env = VecUAVEnv(E, 16, 32, 1, 1, seed=77, full_reset_period=200)
    env.desc.flags = 1
    env.generate_scenes()
    env.reset(episode=1)
    acts = torch.randint(0, 2, (T, E), device=dev, dtype=torch.int8)
    obs = torch.empty(T, E, 5, 14, device=dev)
    rew = torch.empty(T, E, dtype=torch.float64, device=dev)
    done = torch.empty(T, E, dtype=torch.uint8, device=dev)
    info = torch.empty(T, E, 8, dtype=torch.float64, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            env.step(acts if T > 1 else acts[0], obs_out=obs if T > 1 else obs[0], reward_out=rew if T > 1 else rew[0],
                     done_out=done if T > 1 else done[0], info_out=info if T > 1 else info[0])
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(50):
                env.step(acts if T > 1 else acts[0], obs_out=obs if T > 1 else obs[0],
                         reward_out=rew if T > 1 else rew[0], done_out=done if T > 1 else done[0],
                         info_out=info if T > 1 else info[0])
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"T={T}: {e0.elapsed_time(e1) / 200 * 1e3:.2f} us per launch")
