"""bench.py's rank launcher (no GPU): `bench.py --gpus N` started without a
launcher starts N rank processes with the environment torch.distributed.run
would give them, and a process whose launcher world disagrees with --gpus
exits non-zero."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 4, 8])
def test_launcher_starts_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--rank-probe"], env=_env(), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(got) == n
    assert sorted(int(g["RANK"]) for g in got) == list(range(n))
    for g in got:
        assert g["LOCAL_RANK"] == g["RANK"] and g["WORLD_SIZE"] == str(n) and g["MASTER_ADDR"] == "127.0.0.1"
    assert len({g["MASTER_PORT"] for g in got}) == 1


def test_single_gpu_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--rank-probe"], env=_env(), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(got) == 1 and got[0]["WORLD_SIZE"] is None


@pytest.mark.parametrize("gpus,world", [(1, 8), (8, 2), (4, 1)])
def test_world_mismatch_exits_nonzero(gpus, world):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus), "--rank-probe"],
                       env=_env(WORLD_SIZE=str(world), RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "joined a world of %d" % world in r.stderr


def test_failed_rank_fails_the_launch():
    # rank 1 of 4 exits 3: the launch exits 3 and names the rank
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--rank-probe"], env=_env(ZKGPU_BENCH_PROBE_FAIL="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 3
    assert "rank 1 exited with 3" in r.stderr


def test_comm_summary_checks_world():
    sys.path.insert(0, ROOT)
    import bench
    st = {"COUNT_COMM_WORLD": 4.0, "COUNT_COMM_EXCHANGES": 10.0, "COUNT_COMM_BYTES_SENT": 1000.0,
          "COUNT_COMM_MAX_BYTES_SENT": 400.0, "COUNT_COMM_MAX_OPS": 6.0}
    c = bench.comm_summary(st, 4)
    assert c["comm_world"] == 4 and c["rank0_bytes_sent_per_exchange"] == 100 and c["max_ops_per_exchange"] == 6
    assert bench.comm_summary({"STARK_TOTAL": 1.0}, 1) is None
    with pytest.raises(SystemExit):
        bench.comm_summary(st, 8)


def test_shm_outbox_covers_the_largest_exchange():
    """bench.py --comm shm sizes each rank's outbox for its largest message set:
    a commit's return of its column share over the extended rows, or its
    n-domain block of the widest section (the capacities
    tests/test_gpu_sharded_full.py ran the config-4 and zkEVM-shaped proofs with)"""
    import types
    import bench
    args = types.SimpleNamespace(log_n=23, blowup_bits=1)
    c4 = types.SimpleNamespace(n_cm1=100, n_cm2=26, n_cm3=27, n_cm4=6, n_const=30)
    for w, need in ((2, 50 * 2**24 * 8 // 2), (8, 13 * 2**24 * 8 * 7 // 8)):
        b = bench.shm_outbox_bytes(c4, args, w)
        assert need <= b <= 1.3 * need, (w, b, need)
    zk = types.SimpleNamespace(n_cm1=751, n_cm2=168, n_cm3=408, n_cm4=6, n_const=234)
    args20 = types.SimpleNamespace(log_n=20, blowup_bits=1)
    assert bench.shm_outbox_bytes(zk, args20, 8) <= 2 << 30 and bench.shm_outbox_bytes(zk, args20, 2) <= 4 << 30
