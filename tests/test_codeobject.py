"""CPU build-time guard on the code objects of the hot kernels (hipcc cross-compiles gfx950 here).

The one-launch rollout (k_rollout_steps, rollout_steps.hip) keeps the register allocation of the
single-step kernel only because its body launders the thread index and the kernel arguments per step
(left alone, LLVM hoists the loop-invariant lane arithmetic and arguments out of
the step loop and spills 1,412 VGPRs). A compiler change that undoes that would otherwise show up
only as a silent ~10 % loss in a GPU bench. This test compiles the device code to assembly (a few
seconds) and checks, from the amdhsa metadata and the kernel body:
  * spills: VGPR spill count at most 32, SGPR at most 8 (today 14 / 8; the LICM failure mode spills 1,412),
  * LDS: the fixed group segment fits gfx950's 160 KiB,
  * VGPRs: at most 256 (two waves per SIMD at 512 threads),
  * MFMA issue: the counts of v_mfma_f32_16x16x4_f32 and of the split products'
    v_mfma_f32_16x16x32_f16 in the body (the GEMM structure; a change here is a structural change
    of the kernel and must come with DESIGN.md).
The training and single-step policy kernels get the spill / LDS / VGPR part of the same check."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "target-allocation-ppo-transformer_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950", "-I" + os.path.join(ROOT, "include"),
         "-Wno-unused-function", "--offload-device-only", "-S"]

pytestmark = pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="needs hipcc")


def compile_asm(src, tmp_path):
    out = tmp_path / (os.path.basename(src) + ".s")
    subprocess.run([HIPCC] + FLAGS + [os.path.join(CSRC, src), "-o", str(out)], check=True, cwd=CSRC,
                   capture_output=True, timeout=600)
    return out.read_text()


def kernels(asm):
    """{mangled name: metadata dict (ints)} from the amdhsa.kernels YAML."""
    meta = asm[asm.index("amdhsa.kernels:"):]
    out = {}
    for blk in meta.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        out[name] = {k: int(re.search(r"\.%s:\s+(\d+)" % k, blk).group(1))
                     for k in ("vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "group_segment_fixed_size")}
    return out


def body(asm, name):
    i = asm.index("\n" + name + ":")
    return asm[i:asm.index(".Lfunc_end", i)]


# (f32, f16) MFMA instructions in k_rollout_steps: the f32 GEMMs (embeddings -- the critic's five
# positions, the actor's position 4 -- and heads) and the split-product GEMMs of every encoder layer
# 
ROLLOUT_MFMA = (88, 636)


def check_limits(name, m, vgpr_spills=32, sgpr_spills=8):
    print(f"{name}: {m}")
    assert m["vgpr_spill_count"] <= vgpr_spills, (name, m)
    assert m["sgpr_spill_count"] <= sgpr_spills, (name, m)
    assert m["group_segment_fixed_size"] <= 160 * 1024, (name, m)
    assert m["vgpr_count"] <= 256, (name, m)


def test_rollout_steps_code_object(tmp_path):
    asm = compile_asm("rollout_steps.hip", tmp_path)
    ks = kernels(asm)
    name = next(k for k in ks if "k_rollout_stepsILi1E" in k)  # the two-envs-per-wave instantiation (bench)
    check_limits(name, ks[name])
    b = body(asm, name)
    n_f32 = len(re.findall(r"\bv_mfma_f32_16x16x4_f32\b", b))
    n_f16 = len(re.findall(r"\bv_mfma_f32_16x16x32_f16\b", b))
    print(f"{name}: {n_f32} v_mfma_f32_16x16x4_f32, {n_f16} v_mfma_f32_16x16x32_f16 (split products)")
    assert (n_f32, n_f16) == ROLLOUT_MFMA


def test_policy_kernels_code_objects(tmp_path):
    ks = kernels(compile_asm("policy.hip", tmp_path))
    wanted = {"k_policy_backward": 0, "k_policy_forwardILb1ELb0ELi0E": 0, "k_policy_forwardILb0ELb1ELi3E": 0,
              "k_policy_forwardILb0ELb0ELi0E": 0, "k_policy_forwardILb0ELb1ELi0ELb1E": 0}
    for frag in wanted:
        names = [k for k in ks if frag in k]
        assert names, frag
        for n in names:
            check_limits(n, ks[n], sgpr_spills=48)  # the training forward spills 42 SGPRs to VGPR lanes today


READELF = os.environ.get("READELF", "/opt/rocm/lib/llvm/bin/llvm-readelf")


@pytest.mark.skipif(not os.path.exists(READELF), reason="needs llvm-readelf")
def test_rollout_steps_carries_one_env_path(tmp_path):
    """k_rollout_steps is instantiated per env-step path (policy.hip kEnvGrp / kEnvWave): with both
    paths compiled in it was 71 KB of code and spilled 28 VGPRs; the grouped instantiation the bench
    runs is 58.5 KB (62 KB since round 5's range scaling). Guard on its code size, so both paths do not
    creep back into one kernel."""
    out = tmp_path / "rs.o"
    subprocess.run([HIPCC] + [f for f in FLAGS if f != "-S"] + ["--no-gpu-bundle-output", "-c",
                   os.path.join(CSRC, "rollout_steps.hip"), "-o", str(out)], check=True, cwd=CSRC,
                   capture_output=True, timeout=600)
    syms = subprocess.run([READELF, "-sW", str(out)], check=True, capture_output=True, text=True).stdout
    sizes = {l.split()[7]: int(l.split()[2]) for l in syms.splitlines() if " FUNC " in l and "k_rollout_steps" in l}
    print(sizes)
    grp = next(v for k, v in sizes.items() if "k_rollout_stepsILi1E" in k)
    assert grp <= 65 * 1024, sizes
