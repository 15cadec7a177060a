"""CPU plumbing of the library-owned RCCL communicator (include/ptzba.h ptzba_comm_*, csrc/comm.cpp): RCCL is
loaded at run time, so PTZBA_RCCL_LIB can point libptzba at a test double (tests/stubs/stub_rccl.c, built
here with gcc).  Checks the unique-id hand-off, rank / world passing, the fp64-sum all-reduce call, the split
and the error path -- no GPU.  The real RCCL path runs on the GPU box (tests/test_gpu_distributed.py)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "pan-tilt-zoom-slam_amd")

SCRIPT = r'''
import sys, numpy as np
sys.path.insert(0, {pkg!r})
import ptzba
uid = ptzba.Comm.unique_id()
assert uid.startswith(b"stub-rccl-unique-id") and len(uid) == ptzba.UNIQUE_ID_BYTES, uid
c = ptzba.Comm(uid, rank=1, world=3, device=-1)
x = np.arange(5, dtype=np.float64)
c.allreduce(x.ctypes.data, len(x))          # the stub sums 3 identical contributions
assert np.array_equal(x, 3 * np.arange(5)), x
assert c.info() == (1, 3), c.info()
g = c.split(color=1, key=1)
assert g.info() == (1, 2) and (g.rank, g.world) == (1, 2), g.info()   # reported by RCCL for the new comm
y = np.ones(4)
g.allreduce(y.ctypes.data, 4)
assert np.array_equal(y, 2 * np.ones(4)), y   # the stub's split keeps (3 + 1) // 2 ranks
g.close(); c.close()
try:
    ptzba.Comm(b"not-a-stub-id".ljust(128, b"\0"), rank=0, world=2, device=-1)
    raise SystemExit("bad id accepted")
except ptzba.PtzbaError as e:
    assert "ncclCommInitRank" in str(e) and "invalid argument (stub)" in str(e), e
try:
    ptzba.Comm(uid, rank=2, world=2, device=-1)
    raise SystemExit("bad rank accepted")
except ptzba.PtzbaError as e:
    assert "bad communicator arguments" in str(e), e
print("comm plumbing ok")
'''


def _build_stub(tmp_path):
    so = os.path.join(tmp_path, "libstub_rccl.so")
    subprocess.run(["gcc", "-O1", "-shared", "-fPIC", os.path.join(HERE, "stubs", "stub_rccl.c"), "-o", so], check=True)
    return so


def test_comm_plumbing_with_stub_rccl(tmp_path):
    so = _build_stub(str(tmp_path))
    env = dict(os.environ, PTZBA_RCCL_LIB=so)
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(pkg=PKG)], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0 and "comm plumbing ok" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_comm_reports_missing_rccl(tmp_path):
    env = dict(os.environ, PTZBA_RCCL_LIB=os.path.join(str(tmp_path), "no_such_librccl.so"))
    code = (f"import sys; sys.path.insert(0, {PKG!r}); import ptzba\n"
            "try:\n    ptzba.Comm.unique_id()\nexcept ptzba.PtzbaError as e:\n    print('ERR', e)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert "ERR" in r.stdout and "RCCL not available" in r.stdout, (r.stdout, r.stderr[-2000:])
