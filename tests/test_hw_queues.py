"""CPU: the package sets HIP's hardware-queue count before HIP initialises
when the environment leaves it unset, and honours an exported value unless
MXD_HW_QUEUES explicitly asks for more (mlx_data_amd/__init__.py; DESIGN.md
section 7: the prefetch workers' device calls serialise over HIP's default 4
queues; ADVICE r4: an exported setting is the user's)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = ("import os, sys; sys.path.insert(0, %r); import mlx_data_amd; "
         "print(os.environ.get('GPU_MAX_HW_QUEUES', 'unset'))" % os.path.join(REPO, "mlx-data_amd"))


def queues_after_import(**env):
    e = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "MXD_HW_QUEUES")}
    e.update(env)
    r = subprocess.run([sys.executable, "-c", PROBE], env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip().splitlines()[-1]


@pytest.mark.parametrize("env, want", [
    ({}, "16"),                                                  # unset -> package default
    ({"GPU_MAX_HW_QUEUES": "4"}, "4"),                           # exported -> the user's setting wins
    ({"GPU_MAX_HW_QUEUES": "24"}, "24"),
    ({"MXD_HW_QUEUES": "8", "GPU_MAX_HW_QUEUES": "4"}, "8"),    # explicit opt-in raises (and logs)
    ({"MXD_HW_QUEUES": "8", "GPU_MAX_HW_QUEUES": "24"}, "24"),  # never lowered
    ({"MXD_HW_QUEUES": "64"}, "32"),                             # clamped to 32
    ({"MXD_HW_QUEUES": "0", "GPU_MAX_HW_QUEUES": "4"}, "4"),     # 0 leaves HIP's setting alone
    ({"MXD_HW_QUEUES": "0"}, "unset"),
])
def test_hw_queue_policy(env, want):
    assert queues_after_import(**env) == want
