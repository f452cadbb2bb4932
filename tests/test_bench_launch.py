"""CPU: `bench.py --gpus N` starts its own N ranks when no launcher did
(torch.distributed.run on 127.0.0.1, as a child process), and refuses a
WORLD_SIZE that disagrees with --gpus.  gloo, no GPU work (--selftest-launch)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_bench_starts_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--selftest-launch", "--backend", "gloo"], capture_output=True, text=True,
                       env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    doc = json.loads(line)
    assert doc["launch_selftest"] and doc["n_gpus"] == 2 and doc["ranks"] == [0, 1]
    # the per-rank diagnosis the N > 1 lines carry (bench.rank_diag)
    diag = doc["rank_diag"]
    assert [d["rank"] for d in diag] == [0, 1]
    for d in diag:
        assert set(d) == {"rank", "compute_ms", "gather_ms", "gather_bytes"}
        assert d["compute_ms"] > 0 and d["gather_ms"] > 0
    assert diag[0]["gather_bytes"] == 2 * 4096 * 4 and diag[1]["gather_bytes"] == 4096 * 4


def test_bench_refuses_world_mismatch():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--selftest-launch"], capture_output=True, text=True,
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_bench_refuses_instrumented_library():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--legs", "none"],
                       capture_output=True, text=True, env=_env(SALN_LIB="/tmp/x.so"), timeout=120)
    assert r.returncode != 0 and "SALN_LIB" in r.stderr


def test_bench_refuses_leftover_experiment_variables():
    """Any SALN_* variable outside bench.py's allow-list (empty: the engine
    reads none; its tuning goes through saln_option_set) stops the bench
    before it touches the GPU, naming the variable."""
    for var in ("SALN_PK_STEADY", "SALN_ROWS_K", "SALN_ANYTHING"):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--legs", "none"],
                           capture_output=True, text=True, env=_env(**{var: "0"}), timeout=120)
        assert r.returncode != 0 and var in r.stderr, (var, r.stderr[-500:])
    sys.path.insert(0, ROOT)
    import bench
    assert bench.refused_env({"SALN_X": "1", "PATH": "/bin", "XSALN_Y": "2"}) == ["SALN_X"]
    assert bench.refused_env({k: "1" for k in bench.ALLOWED_ENV}) == []
