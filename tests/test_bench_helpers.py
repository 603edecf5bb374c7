"""bench.py's evidence plumbing on the CPU (no GPU): the PMC summary lookup matches rocprofv3's
template-instance kernel names (roofline.traffic was null because k_rollout_steps<1> did
not match), the env step's traffic is dropped when it implies more than the HBM peak at the measured
time, and the weight-stream view prices one weight read per workgroup and step."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "target-allocation-ppo-transformer_amd"))


@pytest.fixture
def bench(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    import bench as b
    return b


def test_kernel_base_strips_namespaces_and_templates(bench):
    assert bench._kernel_base("uavhip::pol::k_rollout_steps<1>") == "k_rollout_steps"
    assert bench._kernel_base("k_policy_forward<false, true, true>") == "k_policy_forward"
    assert bench._kernel_base("uavhip::k_gae") == "k_gae"


def test_profiled_traffic_matches_template_instances(bench, tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r99_pmc.json").write_text(json.dumps({"pmc": {
        "uavhip::pol::k_rollout_steps<1>": {"hbm_bytes_per_launch": 123.0},
        "uavhip::k_env_step<1, false>": {"hbm_bytes_per_launch": 7.0}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.profiled_traffic("k_rollout_steps") == (123.0, "r99_pmc.json")
    assert bench.profiled_traffic("k_env_step<1, false>") == (7.0, "r99_pmc.json")  # the exact name first
    assert bench.profiled_traffic("k_missing") == (None, None)


def test_profiled_traffic_refuses_ambiguous_template_matches(bench, tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r99_pmc.json").write_text(json.dumps({"pmc": {
        "uavhip::pol::k_rollout_steps<1>": {"hbm_bytes_per_launch": 1.0},
        "uavhip::pol::k_rollout_steps<2>": {"hbm_bytes_per_launch": 2.0}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.profiled_traffic("k_rollout_steps") == (None, None)


def test_env_share_reads_the_newest_summary(bench, tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r98_env_share.json").write_text(json.dumps({"env_bytes_per_step": 1.0, "env_ns_per_step": 10.0}))
    (prof / "r99_env_share.json").write_text(json.dumps({"env_bytes_per_step": 2.0, "env_ns_per_step": 20.0}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.env_share_traffic() == (2.0, "r99_env_share.json", 20.0)


def test_weight_stream_prices_one_weight_read_per_workgroup_step(bench):
    from uavhip._lib import LIB
    n = int(LIB.uavhip_policy_layout(None, 0))
    w = bench.weight_stream(0.05, 4096)
    assert w["workgroups"] == 256 and w["bytes_per_workgroup_step"] == 4 * n
    assert abs(w["achieved"] - 4 * n * 256 / 50e-6 / 1e9) < 1e-6
    assert abs(w["frac"] - w["achieved"] / bench.L2_PEAK_GBS) < 1e-12


def test_env_traffic_dropped_when_it_exceeds_the_hbm_peak(bench):
    # round 3's line: 70.9 MB per step against a 2.56 us time = 27.7 TB/s -> dropped, with the reason
    t, gbs, ok, why = bench.check_traffic(70.9e6, 2.56e-3)
    assert t is None and ok is False and gbs > bench.HBM_PEAK_GBS and "HBM peak" in why
    t, gbs, ok, why = bench.check_traffic(9.4e6, 3.0e-3)  # round 4: 9.4 MB over 3.0 us = 3.1 TB/s
    assert t == 9.4e6 and ok is True and why is None and abs(gbs - 3133.3) < 1
    assert bench.check_traffic(None, 1.0) == (None, None, None, None)
