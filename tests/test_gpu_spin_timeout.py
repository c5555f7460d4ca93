"""Generation-word timeouts are loud (VERDICT r04 Next 3).

The wave-specialised dual GEMM (ctn_dual_ws.hip, on by default in every TemporalBlock
backward) hands tiles between its memory, row and column waves through LDS generation
words, and every wait on them is bounded.  A wait that runs out sets CTN_DEVERR_SPIN in the
device error word; the host reports it (ctn_device_status, and ctn_tblock_reduce_grads at
the next backward pass) as CTN_ERR_HIP, so a protocol error can neither hang the GPU nor
corrupt gradients silently.

The debug library libctn_hip_spin1.so (Makefile: CTN_SPIN_LIMIT=1, every wait gives up
after one poll) takes the timeout path in the first launch; a block backward through it
must report the error, and the default library must not.  Each library runs in a child
process (one CDLL per process).  GPU only.
"""
import os
import subprocess
import sys

import pytest

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import ctypes, sys, torch
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {tests!r})
import ctn_lib as L
from test_gpu_benchshape import _block_params, _hip_block
torch.manual_seed(0)
params = _block_params(3, 256, 512)
x = torch.randn(4, 256, 3199)
G = torch.randn(4, 256, 3199)
_hip_block(x, G, params, 2, 0, "gLN", torch.bfloat16, packed=True)
lib = L.load()
w = ctypes.c_uint32(0)
rc = lib.ctn_device_status(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), ctypes.byref(w), 1)
msg = lib.ctn_last_error().decode() if rc else ""
w2 = ctypes.c_uint32(7)
rc2 = lib.ctn_device_status(None, ctypes.byref(w2), 0)      # cleared by the first call
print("RESULT", rc, w.value, rc2, w2.value, msg, flush=True)
"""


def _run(lib_name):
    env = dict(os.environ, CTN_HIP_LIB=os.path.join(PKG, lib_name))
    code = SCRIPT.format(pkg=PKG, tests=os.path.join(ROOT, "tests"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT")][-1].split(" ", 5)
    return int(line[1]), int(line[2]), int(line[3]), int(line[4]), line[5] if len(line) > 5 else ""


@pytest.mark.timeout(400)
def test_forced_timeout_is_reported():
    if not os.path.exists(os.path.join(PKG, "libctn_hip_spin1.so")):
        pytest.fail("libctn_hip_spin1.so not built (make)")
    rc, word, rc2, word2, msg = _run("libctn_hip_spin1.so")
    assert rc == 4 and word & 1, (rc, word, msg)          # CTN_ERR_HIP, CTN_DEVERR_SPIN
    assert "CTN_DEVERR_SPIN" in msg, msg
    assert rc2 == 0 and word2 == 0, (rc2, word2)          # clear=1 reset the word


@pytest.mark.timeout(400)
def test_default_library_reports_no_error():
    rc, word, rc2, word2, msg = _run("libctn_hip.so")
    assert rc == 0 and word == 0, (rc, word, msg)
