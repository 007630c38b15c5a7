"""The GICP help board (built by -DPCORE_GICP_HELP_BOARD=1, off in the default build, where
these tests check that nothing is enlisted): once gicp_kernel's pose queue runs dry, the waves that find it empty
search correspondences for the poses still being refined.  A helper's round is the owner's own search on the
same published float transform, so every output is bit-identical with the board off (PCORE_GICP_HELP=0) -- checked
here on a batch smaller than the resident waves (the queue is dry from the start: every multi-round pose is helped
from its first iterations) and on C3's full 50k batch (help only in the launch's tail)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from perception_amd import workloads

pytestmark = pytest.mark.gpu

C3_NAMES = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]


def _run(w, monkeypatch, help_on):
    if help_on:
        monkeypatch.delenv("PCORE_GICP_HELP", raising=False)
    else:
        monkeypatch.setenv("PCORE_GICP_HELP", "0")
    outs = w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
    outs = [o.cpu().numpy() for o in outs]
    return outs, w.core.stats(), w.core.gicp_help_stats()


@pytest.mark.parametrize("per_model", [300, 10000])
def test_help_board_outputs_equal_help_off(per_model, monkeypatch):
    w = workloads.build(names=C3_NAMES, poses_per_model=per_model)
    on, st_on, hs = _run(w, monkeypatch, True)
    off, st_off, hs_off = _run(w, monkeypatch, False)
    for a, b in zip(on, off):
        assert np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))
    assert st_on["gicp_iterations"] == st_off["gicp_iterations"]
    assert st_on["gicp_iterations_run"] == st_off["gicp_iterations_run"]
    assert hs_off == {"helper_rounds": 0, "owner_timeouts": 0, "helper_giveups": 0, "poses_enlisted": 0}
    if hs == hs_off:
        pytest.skip("the library is built without the help board (PCORE_GICP_HELP_BOARD=0)")
    # the board was used: poses enlisted and rounds searched by helpers
    assert hs["poses_enlisted"] > 0 and hs["helper_rounds"] > 0, hs
    print("help board", per_model, hs)
