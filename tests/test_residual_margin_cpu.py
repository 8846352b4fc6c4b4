"""How far the stopping decisions sit from their thresholds.

OpenCV 3.4.1's procOneScale stops a warp from cuda::sum of the float diff buffer (behind
/root/reference/src/optflow.cpp:518-519).  Its accumulation type and order are recalled,
not verified [OCV], so the oracle's double, in-order sum might decide a check differently
from the reference's.  These tests pin, on the golden fixtures (tests/golden/):
  * every check's error / scaledEps is at least MIN_MARGIN (relative) away from each
    threshold that could change the schedule (1 for stop / continue, then 2, 4, 6, ... for
    when the next check comes: oracle.checker.check_margins);
  * a different, lossy accumulation (float rows, float total, rows reversed) gives the same
    per-warp iteration counts, and its residuals stay within a factor SAFETY of those
    margins.
The C2 / C3 / production-strip figures are in profiles/r4/residual_margins.md
(tests/analysis/residual_margins.py)."""
import json
from pathlib import Path

import numpy as np
import pytest

from optflow_amd import capi
from oracle import checker

GOLDEN = sorted((Path(__file__).resolve().parent / "golden").glob("*.npz"))
MIN_MARGIN = 1e-4   # measured minimum over the fixtures: 5.1e-4
SAFETY = 100        # measured: >= 960x between the margin and the float-vs-double deviation


def params_of(d):
    pj = json.loads(str(d["params"]))
    return capi.make_params(**{k: v for k, v in pj.items() if k in capi.DEFAULTS})


@pytest.mark.parametrize("f", GOLDEN, ids=[f.stem for f in GOLDEN])
def test_checks_clear_of_thresholds_and_float_accumulation_keeps_schedule(built, f):
    d = np.load(f)
    p = params_of(d)
    u, v, st, wi, tr = checker.oracle_check_trace(d["I0"], d["I1"], p)
    np.testing.assert_array_equal(wi, d["warp_iters"])      # the trace does not perturb
    assert st["checks_total"] == len(tr)
    if p.epsilon == 0:                                     # fixed work: no checks at all
        assert len(tr) == 0
        return
    m = checker.check_margins(tr, p.iterations)
    assert m.min() >= MIN_MARGIN, tr[np.argmin(m)]
    u1, v1, _, wi1, tr1 = checker.oracle_check_trace(d["I0"], d["I1"], p, residual_mode=1)
    np.testing.assert_array_equal(wi1, wi)
    assert np.array_equal(u1.view(np.uint32), u.view(np.uint32))   # same schedule => same bits
    assert np.array_equal(tr1[:, :3], tr[:, :3])
    dev = np.abs(tr1[:, 3] / tr[:, 3] - 1.0)
    assert dev.max() > 0                                   # the accumulation did change
    assert dev.max() * SAFETY <= m.min()


def test_margin_thresholds_follow_procOneScale():
    """check_margins' thresholds: stop iff r <= 1; the next check comes 2 iterations later
    iff r < 2, 4 later iff r < 4, ...; only thresholds reachable before `iterations`."""
    tr = np.array([[0, 0, 1, 1.5], [0, 0, 3, 2.02], [0, 0, 5, 3.9], [0, 0, 295, 7.0]])
    m = checker.check_margins(tr, 300)
    np.testing.assert_allclose(m, [0.5 / 1.5, 0.02 / 2.02, 0.1 / 3.9, 3.0 / 7.0])   # 6 is out of reach at n = 295
