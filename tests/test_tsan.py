"""The host scheduler under ThreadSanitizer (VERDICT r1 weak
11): tests/native/sched_stress.cpp -- Prefetch / OrderedPrefetch / ThreadPool
over shared streams and buffers, set_state churn against drawing workers,
shared arrays batched from many threads, and a Prefetch /
OrderedPrefetch whose last reference is released by one of its own pool's
tasks with others still queued, at one and four workers (the pre-fix code
deadlocks or aborts with EDEADLK there; the stress binary fails fast on it) --
compiled with -fsanitize=thread
together with the pipeline sources and run on the CPU.  Any race report fails
the test (halt_on_error)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mlx-data_amd")


def test_scheduler_is_race_free_under_tsan():
    b = subprocess.run(["make", "-s", "-C", PKG, "tsan"], capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1")
    r = subprocess.run([os.path.join(PKG, "build", "tsan", "sched_stress")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0, r.stderr[-3000:]
    assert "sched_stress: ok" in r.stdout
