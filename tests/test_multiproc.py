"""apex.parallel.multiproc (R-19): argv injection, env, rank-0 stdout, failure propagation."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, time
r = int(os.environ["RANK"]); w = int(os.environ["WORLD_SIZE"])
assert sys.argv[sys.argv.index("--rank") + 1] == str(r)
assert sys.argv[sys.argv.index("--world-size") + 1] == str(w)
assert os.environ["MASTER_ADDR"] == "127.0.0.1"
if "--fail" in sys.argv:
    if r == 1:
        sys.exit(3)
    time.sleep(60)
print("child-ok", r, w)
'''


def _run(tmp_path, extra):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-m", "apex.parallel.multiproc", "--nproc", "3", str(script)] + extra,
                          cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120)


def test_multiproc_launch(tmp_path):
    r = _run(tmp_path, [])
    assert r.returncode == 0, r.stderr
    assert "child-ok 0 3" in r.stdout
    assert "child-ok 2 3" in (tmp_path / "GPU_2.log").read_text()


def test_multiproc_failure_propagates(tmp_path):
    t0 = time.time()
    r = _run(tmp_path, ["--fail"])
    assert r.returncode == 3
    assert time.time() - t0 < 50  # siblings were terminated, not waited for
