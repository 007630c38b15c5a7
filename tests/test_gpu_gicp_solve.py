"""The GICP kernels' damped LM solve on the GPU (gicpm::lm_solve_schur, uniform on the wave, through
pcore_debug_lm_solve) against the oracle's host build of the same function (held to numpy's dense solve by
tests/test_gicp_spec.py), bit for bit on the same 4,000+ random SPD and indefinite, tied, zero and non-finite systems:
the fused products (fma) and IEEE divisions round identically on both sides."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle  # noqa: E402
from perception_amd import _native  # noqa: E402
from tests.test_gicp_spec import lm_solve_cases  # noqa: E402

pytestmark = pytest.mark.gpu


def _same(a, b):
    """Bit-identical, NaNs compared by position (their payloads are not the arithmetic's)."""
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(np.where(na, 0.0, a).view(np.uint64),
                                                     np.where(nb, 0.0, b).view(np.uint64))


def test_gpu_lm_solve_equals_oracle_bitwise():
    cases = lm_solve_cases()
    sys_h = np.stack([c[0] for c in cases]).astype(np.float64)
    lam_h = np.array([c[1] for c in cases], np.float64)
    n = len(cases)
    dev = torch.device("cuda", 0)
    sys_d = torch.from_numpy(sys_h).to(dev)
    lam_d = torch.from_numpy(lam_h).to(dev)
    out = torch.full((n, 6), float("nan"), dtype=torch.float64, device=dev)
    lib = _native.load()
    rc = lib.pcore_debug_lm_solve(sys_d.data_ptr(), lam_d.data_ptr(), out.data_ptr(), n, None)
    assert rc == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    bad = [i for i in range(n) if not _same(got[i], oracle.gicp_lm_solve_sys(sys_h[i], lam_h[i]))]
    assert not bad, (len(bad), bad[:5])
