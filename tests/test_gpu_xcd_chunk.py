"""The XCD-chunked tile slots (modem_device.h xcd_slot / xcd_chunk, round 6) only decide which
workgroup runs which tile: every tile is still computed once, by the same code. The samples, I/Q
and decisions of two consecutive steps of C3's chain (one channel, 2^24 samples: a persistent grid
that is a multiple of 64, so the chunk applies) and of an 8-channel batch chain (C4's shape, 2^22
samples per channel, 128 workgroups per channel) are bit-identical with MODEM_XCD_CHUNK = 1 (the
plain grid-strided walk), 8 (the default) and 16. One subprocess per setting: the switch is read
once per process. Reference: modulator.rs:64-101, demodulator.rs:44-56 (one stream per handle; the
schedule is not part of the result)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import hashlib, json, sys
sys.path.insert(0, sys.argv[1])
import bench
out = {}
wls = (("c3", bench.WORKLOADS["c3"], False, 0),
       ("batch8", ("qpsk", 2, 65, 4, 1 << 22, 8, 0, "8 x 2^22 QPSK"), True, 8))
for tag, wl, batch, group in wls:
    r = bench.GpuRunner(wl, 0, 0, batch=batch, group=group)
    r.step()
    r.step()
    r.sync()
    h = hashlib.sha256()
    for d in r.ch:
        for k in ("y", "oiq", "osym"):
            h.update(d[k].cpu().numpy().tobytes())
    out[tag] = h.hexdigest()
    del r
print(json.dumps(out))
"""


def _digests(chunk):
    env = dict(os.environ, MODEM_XCD_CHUNK=str(chunk))
    res = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], env=env, capture_output=True, text=True,
                         timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    return json.loads([ln for ln in res.stdout.splitlines() if ln.startswith("{")][-1])


def test_results_do_not_depend_on_the_xcd_chunk():
    base = _digests(1)
    for c in (8, 16):
        assert _digests(c) == base, f"MODEM_XCD_CHUNK={c}"
