"""bench.py's multi-GPU launch contract (the driver's `bench.py --gpus N`), checked
without a GPU: every refusal happens before anything touches one.

* `--gpus N` without torchrun's environment starts the N ranks itself (torch.distributed.run as a
  child process) — unless fewer than N GPUs are visible: RCCL rejects two ranks on one GPU
  ("Duplicate GPU detected"), and a line from fewer ranks would misreport n_gpus, so it refuses
  (exit 3) instead of timing one process;
* under torchrun, WORLD_SIZE must equal --gpus (exit 2 otherwise).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "NERF_DIST_BACKEND")}
    e.update(env)
    e["HIP_VISIBLE_DEVICES"] = e.get("HIP_VISIBLE_DEVICES", "")
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=300)


def test_gpus_more_than_visible_refuses():
    r = _bench(["--gpus", "2", "--no-cpu-baseline"], HIP_VISIBLE_DEVICES="")
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "refusing" in r.stderr and "Duplicate GPU" in r.stderr
    assert r.stdout.strip() == ""          # no bench line from fewer ranks


def test_world_size_must_match_gpus():
    r = _bench(["--gpus", "2", "--no-cpu-baseline"], WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE=3" in r.stderr
