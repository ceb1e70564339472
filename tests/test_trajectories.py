"""Waypoint generators (utils/trajectories.py) against golden vectors generated from the
reference's own utils/trajectories.py (tools/gen_golden.py --only golden_trajectories.npz)."""
import numpy as np

from uav_reinforcement_learning_control_amd.utils import trajectories as T


def test_generators_match_reference_goldens(golden_dir):
    g = np.load(f"{golden_dir}/golden_trajectories.npz")
    for name in ("eight", "circle", "square"):
        for sp in (0.2, 0.5, 0.8):
            ref = g[f"{name}_s{sp}"]
            got = T.make_trajectory(name, spacing=sp)
            assert got.shape == ref.shape, (name, sp)
            np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12)
    np.testing.assert_allclose(T.figure_eight(0.3, 1.5, np.array([0.5, -0.2, 1.2])), g["eight_r1.5_c"], atol=1e-12)
    np.testing.assert_allclose(T.circle(0.3, 0.7, np.array([0.1, 0.2, 0.8])), g["circle_r0.7_c"], atol=1e-12)
    np.testing.assert_allclose(T.square(0.3, 2.0, np.array([-0.3, 0.0, 1.5])), g["square_l2_c"], atol=1e-12)
