"""CPU: ``bench.py --gpus N`` launches N ranks itself (one process per GPU, 127.0.0.1 rendezvous)
when it is not already under torch.distributed, and the ranks meet (gloo dry run, world 2)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_launch_command(monkeypatch):
    import bench
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 0

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.main(["--gpus", "4", "--steps", "3", "--warmup", "1"]) == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-7:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "3", "--warmup", "1"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_dry_run_two_ranks_gloo():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks"] == [0, 1] and d["gpus_arg"] == 2


def _dry(config, world):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dry-run",
                        "--config", config], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_dry_run_c3_partitions_the_node_round():
    """C3 (BASELINE configs[2]): one node round of 1,000 certificates x 667 votes split over the ranks
    (strong scaling), contiguous and complete."""
    d = _dry("C3", 2)
    assert d["config"] == "C3" and d["scaling"] == "strong" and d["total_sigs"] == 1000 * 667
    sh = d["shards"]
    assert sh[0]["first_cert"] == 0 and sh[1]["first_cert"] == sh[0]["ncerts"]
    assert sum(s["ncerts"] for s in sh) == 1000 and sum(s["sigs"] for s in sh) == 667000
    assert all(s["digest_batches"] == 0 for s in sh)


def test_dry_run_c4_per_rank_shape_with_digests():
    """C4 (BASELINE configs[3]): every rank verifies 1,250 x 6,667 and digests its 1,250 worker
    batches inside the step (weak scaling); global certificate indices do not overlap."""
    d = _dry("C4", 2)
    assert d["config"] == "C4" and d["scaling"] == "weak" and d["total_sigs"] == 2 * 1250 * 6667
    assert [s["first_cert"] for s in d["shards"]] == [0, 1250]
    assert all(s["ncerts"] == 1250 and s["sigs"] == 1250 * 6667 and s["digest_batches"] == 1250
               for s in d["shards"])


def test_config_plan_single_rank():
    import argparse
    import bench
    args = bench.parse_args(["--config", "C3"])
    p = bench.config_plan(args, 1, 0)
    assert (p["first_cert"], p["ncerts"], p["votes"], p["validators"]) == (0, 1000, 667, 1000)
    args = bench.parse_args([])
    p = bench.config_plan(args, 8, 3)
    assert (p["first_cert"], p["ncerts"], p["votes"], p["total_sigs"]) == (3 * 14926, 14926, 67, 8 * 14926 * 67)
    assert isinstance(args, argparse.Namespace)


def test_fm_work_model_matches_kernel_chain():
    """k_verify executes 7 FM per comb position except the chain's first entry (1 FM) and its last
    addition (6 FM, no T): C2 (W24 basepoint, W20 keys) = 7 x (11 + 13 - 1) + 1 - 1 = 161."""
    import bench
    assert bench.kverify_fm_per_sig(20, 24) == 161
    assert bench.kverify_fm_per_sig(16, 24) == 7 * (11 + 16 - 1)
