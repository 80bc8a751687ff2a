"""bench.py --gpus N: the launcher that runs N RCCL ranks without an external torchrun.

A stub target stands in for the bench (no GPU here): it records the environment each child gets and
exits with a chosen code, so the test pins the per-rank variables (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT), the exit-code propagation (the failing child's code, the others
terminated) and the refusal to time fewer GPUs than asked."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

STUB = r'''
import json, os, sys, time
out = os.environ["STUB_DIR"]
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
json.dump({"env": {k: os.environ.get(k) for k in keys}, "argv": sys.argv[1:]},
          open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w"))
rank = int(os.environ["RANK"])
fail = os.environ.get("STUB_FAIL_RANK")
if fail is not None and int(fail) == rank:
    sys.exit(int(os.environ["STUB_FAIL_RC"]))
if fail is not None:
    time.sleep(120)           # the healthy ranks would wait in a collective: the launcher must end them
'''


def _stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return str(p)


def test_launcher_env_per_rank(tmp_path):
    env = dict(os.environ, STUB_DIR=str(tmp_path))
    env.pop("STUB_FAIL_RANK", None)
    rc = bench.launch_ranks(4, ["--gpus", "4", "--steps", "2"], script=_stub(tmp_path), gpus=8, env=env)
    assert rc == 0
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(4)]
    ports = {r["env"]["MASTER_PORT"] for r in recs}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, rec in enumerate(recs):
        e = rec["env"]
        assert e["RANK"] == str(r) and e["LOCAL_RANK"] == str(r), e
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4", e
        assert e["MASTER_ADDR"] == "127.0.0.1", e
        assert rec["argv"] == ["--gpus", "4", "--steps", "2"]


def test_launcher_propagates_failing_rank_and_ends_the_others(tmp_path):
    env = dict(os.environ, STUB_DIR=str(tmp_path), STUB_FAIL_RANK="1", STUB_FAIL_RC="3")
    t0 = time.time()
    rc = bench.launch_ranks(3, [], script=_stub(tmp_path), gpus=3, env=env)
    assert rc == 3
    assert time.time() - t0 < 60          # the sleeping ranks were terminated, not waited for


def test_launcher_refuses_fewer_gpus_than_asked(tmp_path):
    env = dict(os.environ, STUB_DIR=str(tmp_path))
    rc = bench.launch_ranks(2, [], script=_stub(tmp_path), gpus=1, env=env)
    assert rc == 2
    assert not list(tmp_path.glob("rank*.json"))      # no child was started


def test_bench_cli_fails_fast_without_gpus():
    """This container has no GPU: `bench.py --gpus 2` must refuse within seconds (exit 2) instead of
    timing one device, and a torchrun WORLD_SIZE that disagrees with --gpus is refused too."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs 2 visible GPUs" in r.stderr
    env.update(WORLD_SIZE="3", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "disagree" in r.stderr


def test_launcher_sigterm_ends_the_ranks(tmp_path):
    """A launcher terminated from outside (a driver's time limit) terminates its ranks too."""
    import signal
    stub = _stub(tmp_path)
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(2, [], script=%r, gpus=2))" % (ROOT, stub))
    env = dict(os.environ, STUB_DIR=str(tmp_path), STUB_FAIL_RANK="7", STUB_FAIL_RC="1")   # no rank fails: all sleep
    p = subprocess.Popen([sys.executable, "-c", code], env=env)
    for _ in range(300):
        if len(list(tmp_path.glob("rank*.json"))) == 2:
            break
        time.sleep(0.1)
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    p.send_signal(signal.SIGTERM)
    assert p.wait(60) == 128 + signal.SIGTERM
    time.sleep(1)
    import psutil
    alive = [c for c in psutil.process_iter(["cmdline"]) if c.info["cmdline"] and stub in " ".join(c.info["cmdline"])]
    assert not alive, alive
    assert len(recs) == 2
