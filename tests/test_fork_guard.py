"""The boundary's fork-after-initialisation guard (deepfmkit_amd/csrc/fork_guard.h).

The reference's callers fork (fitters.py:421-423, experiments.py:381-384). libdfmi.so records
the pid of the process that first initialised HIP; every entry point called from another pid
(a fork made after that point, which inherits HIP state it cannot use) returns DFMI_ERR_HIP
naming both pids, before any HIP runtime call. CPU tests: the guard's logic through the host
build (tests/hostcheck), and the real library in a forked child on this GPU-less container
(the parent's first call records its pid even though no device answers)."""
import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HC = os.path.join(ROOT, "tests", "hostcheck", "libhostcheck.so")


def _guard(init_pid, cur_pid):
    if not os.path.exists(HC):
        pytest.skip("tests/hostcheck/libhostcheck.so not built")
    hc = ctypes.CDLL(HC)
    hc.hc_fork_guard.argtypes = [ctypes.c_long, ctypes.c_long, ctypes.c_char_p, ctypes.c_int]
    hc.hc_fork_guard.restype = ctypes.c_int
    buf = ctypes.create_string_buffer(1024)
    n = hc.hc_fork_guard(init_pid, cur_pid, buf, len(buf))
    return n, buf.value.decode()


def test_guard_passes_before_init_and_in_the_initialising_process():
    assert _guard(0, 4242) == (0, "")      # not initialised yet: a Pool forked after load works
    assert _guard(4242, 4242) == (0, "")   # the process that initialised HIP


def test_guard_refuses_a_fork_made_after_init_naming_both_pids():
    n, msg = _guard(4242, 4343)  # "initialised" by a fake parent pid, called from another
    assert n > 0
    assert "4242" in msg and "4343" in msg and "fork" in msg


CHILD = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
from deepfmkit_amd import _lib
lib = _lib.load()
lib.dfmi_device_count()                 # first call: records this pid (no device here)
parent = os.getpid()
rc_parent = lib.dfmi_step_timing(0)     # same pid: the guard passes (no device -> NODEV)
pid = os.fork()
if pid == 0:
    rc = lib.dfmi_step_timing(0)
    msg = lib.dfmi_last_error().decode()
    ok = rc == -2 and str(parent) in msg and str(os.getpid()) in msg and "fork" in msg
    os._exit(0 if ok else 3)
_, status = os.waitpid(pid, 0)
print("parent rc", rc_parent, "child exit", os.waitstatus_to_exitcode(status))
sys.exit(0 if rc_parent in (0, -3) and os.waitstatus_to_exitcode(status) == 0 else 1)
"""


def test_library_refuses_calls_from_a_fork_after_init():
    """The real libdfmi.so: the parent's first call records its pid; a child forked after
    that gets DFMI_ERR_HIP (-2) with both pids from an entry point, while the parent's own
    calls pass the guard. Run on the CPU-only container (no GPU is touched by the child)."""
    if os.path.exists("/dev/kfd"):
        pytest.skip("runs on the GPU-less container only (no fork of a GPU-initialised process)")
    if not os.path.exists(os.path.join(ROOT, "deepfmkit_amd", "libdfmi.so")):
        pytest.skip("libdfmi.so not built")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout, r.stderr)
