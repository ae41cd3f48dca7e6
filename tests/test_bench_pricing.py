"""bench.py's per-op roofline pricing (host arithmetic only, no GPU): the fused table step moves the
tables' RAdam bytes from the radam op to the hash backward, and calls that launch one of several
kernel variants per launch (compositing K = 1 / 3) take the mean of their kernels' PMC traffic."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _kernels(**ms):
    return {name: {"launches": n, "avg_ms": t / n, "total_ms": t} for name, (n, t) in ms.items()}


def test_fused_table_step_pricing():
    tables, mlp = 16 * (1 << 19) * 2, 18_688
    units = {"point": 1_048_576, "sample": 1_048_576, "hash_point": 786_432, "bwd_point": 1_048_576,
             "bwd_hash_point": 786_432}
    k = _kernels(nerf_hash_encode_bwd_bin_rows=(2, 0.22), nerf_hash_encode_bwd_owner_step=(1, 0.25),
                 nerf_radam_step=(1, 0.004))
    plain = {o["op"]: o for o in bench.op_rooflines(k, 1, units, tables + mlp)}
    fused = {o["op"]: o for o in bench.op_rooflines(k, 1, units, tables + mlp, fused_elems=tables)}
    assert fused["radam"]["units_per_step"] == mlp
    assert fused["radam"]["algorithmic_bytes"] == 28 * mlp
    assert fused["hash_bwd"]["algorithmic_bytes"] == plain["hash_bwd"]["algorithmic_bytes"] + 24 * tables
    assert fused["hash_bwd"]["fused_table_step_bytes"] == 24 * tables
    assert "fused_table_step_bytes" not in plain["hash_bwd"]
    assert fused["hash_bwd"]["calls"] == {"nerf_hash_encode_bwd_bin_rows": 2, "nerf_hash_encode_bwd_owner_step": 1}


def test_kernel_variants_traffic_is_the_mean(tmp_path, monkeypatch):
    t = {"nerf::composite_fwd_kernel<1>": {"traffic_bytes": 1000.0},
         "nerf::composite_fwd_kernel<3>": {"traffic_bytes": 3000.0}}
    path = tmp_path / "traffic.json"
    path.write_text(json.dumps(t))
    monkeypatch.setattr(bench, "traffic_file", lambda: str(path))
    assert bench.pmc_traffic("nerf_composite_fwd") == 2000.0      # x 2 launches per step = both kernels
    assert bench.pmc_traffic("nerf_composite_bwd") is None         # kernels missing from the summary
    assert bench.base_name("nerf_mlp_fwd_ord") == bench.base_name("nerf_mlp_fwd_q") == "nerf_mlp_fwd"
    assert bench.base_name("nerf_mlp_fwd_h3") == "nerf_mlp_fwd"


def test_merged_compositing_calls_are_priced():
    """The coarse compositing inside the sampler launch and the batched backward count toward the
    compositing ops (their time is the op's; the sampler's bytes are not priced)."""
    units = {"point": 1_048_576, "sample": 1_048_576, "hash_point": 786_432, "bwd_point": 1_048_576,
             "bwd_hash_point": 786_432}
    k = _kernels(nerf_composite_fwd=(1, 0.0104), nerf_composite_sample_fine=(1, 0.0216),
                 nerf_composite_bwd_batch=(1, 0.0171))
    ops = {o["op"]: o for o in bench.op_rooflines(k, 1, units, 0)}
    assert ops["composite_fwd"]["calls"] == {"nerf_composite_fwd": 1, "nerf_composite_sample_fine": 1}
    assert abs(ops["composite_fwd"]["ms_per_step"] - 0.032) < 1e-9
    assert ops["composite_bwd"]["calls"] == {"nerf_composite_bwd_batch": 1}
    assert ops["composite_bwd"]["algorithmic_bytes"] == 40 * units["sample"]
