"""Host logic of the weight-gradient schedules (csrc/wgrad.hpp WgPlan; DESIGN.md 5 `k_wgrad`): the
stream-K and the chunked (XCD-aware) decode of k_wgrad replayed on the host for the problem list of
uavhip_ppo_step at several minibatch sizes -- every (problem, tile, k-slab) unit computed exactly
once, one partial slot per run inside the workspace's slot buffer, and the reduction map naming
exactly each tile's run slots (tests/wgrad_plan_check.cpp). hipcc builds the check here; no GPU call."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
pytestmark = pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="needs hipcc")


def test_wgrad_schedules_cover_every_unit_once(tmp_path):
    exe = tmp_path / "wgrad_plan_check"
    subprocess.run([HIPCC, "-std=c++17", "-O1", "--offload-arch=gfx950",
                    "-I", os.path.join(ROOT, "target-allocation-ppo-transformer_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "wgrad_plan_check.cpp"),
                    "-o", str(exe)], check=True)
    # 64: the reference's minibatch; 256 / 1024: trunk-split sizes; 4096: the bench's; 2048 / 8192 others
    r = subprocess.run([str(exe), "64", "256", "1024", "2048", "4096", "8192"], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok ") == 12
