"""The oracle against the committed golden fixtures (tests/golden/, made by make_golden.py).

Bit-exact: the fixtures are the oracle's own outputs, frozen after the numpy cross-check,
so any drift of the checker (compiler flags, a refactor, glibc) shows up here on the CPU.
"""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, GOLDEN)
import make_golden  # noqa: E402

FILES = sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz"))


@pytest.fixture(scope="module")
def regenerated(o):
    return make_golden.build_fixtures()


def test_fixture_set_complete(regenerated):
    assert sorted(regenerated) == FILES
    total = sum(os.path.getsize(os.path.join(GOLDEN, f)) for f in FILES)
    assert total < 2 << 20                       # small fixtures


@pytest.mark.parametrize("fname", FILES)
def test_oracle_matches_fixture(regenerated, fname):
    with np.load(os.path.join(GOLDEN, fname)) as z:   # allow_pickle stays False
        assert sorted(z.files) == sorted(regenerated[fname])
        for k in z.files:
            a, b = z[k], regenerated[fname][k]
            assert a.dtype == b.dtype and a.shape == b.shape, (fname, k)
            assert a.tobytes() == b.tobytes(), (fname, k)


def test_fixture_decisions_are_the_sent_symbols():
    """Size-independent property of the stored loopbacks: every decision equals the symbol sent."""
    for name in ("c1", "c2", "c3", "c5"):
        with np.load(os.path.join(GOLDEN, f"chain_{name}.npz")) as z:
            bps = int(z["bps"][0])
            for bits, sym in ((z["bits"], z["rx_sym"]), (z["win_bits"], z["win_rx_sym"])):
                sent = bits.reshape(-1, bps).astype(np.int64) @ (1 << np.arange(bps)[::-1])
                assert len(sym) > 0 and np.array_equal(sym, sent[: len(sym)].astype(np.uint8)), name
