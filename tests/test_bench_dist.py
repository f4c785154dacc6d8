"""The bench's multi-process path on CPU: world size 2 over gloo (what
torch.distributed.run sets up on an 8-GPU node, minus the GPU).  Checks the
barrier-bracketed timing, the max over ranks and that `value` counts the
images of every rank (weak scaling, no data-path collective)."""
import json
import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
sys.path.insert(0, {repo!r})
import bench
r = bench.Ranks()
assert r.world == 2 and r.dist is not None
delay = 0.01 * (r.rank + 1)          # rank 1 is the slow one
wall, local = bench.timed_steps(r, lambda i: time.sleep(delay), lambda: None, 5)
line = bench.bench_line("c2", r.world, 256, 5, 1, wall, None, None, None)
print(json.dumps(dict(rank=r.rank, wall=wall, local=local, line=line)), flush=True)
r.close()
"""


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_timing():
    port = free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", CHILD.format(repo=REPO)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e
        outs.append(json.loads(o.strip().splitlines()[-1]))
    outs.sort(key=lambda d: d["rank"])
    slow = max(d["local"] for d in outs)
    for d in outs:
        assert d["wall"] == slow  # both ranks report the max over ranks
    assert outs[1]["local"] >= 5 * 0.02
    line = outs[0]["line"]
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["global_batch"] == 512
    assert abs(line["value"] - 2 * 256 * 5 / slow) < 0.1
    assert line["higher_is_better"] is True


def test_bench_launches_its_own_ranks():
    """`bench.py --gpus 2` with no launcher spawns two rank processes (gloo
    barrier + max-over-ranks); the line counts both ranks' batches."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "4",
                        "--simulate", "0.01"], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 512 and line["config"]["per_gpu_batch"] == 256
    # rank 1 sleeps twice as long: the max over ranks sets the wall time
    assert line["ms_per_step"] >= 20.0
    assert abs(line["value"] - 512 * 4 / (line["ms_per_step"] * 4 / 1e3)) / line["value"] < 0.01
