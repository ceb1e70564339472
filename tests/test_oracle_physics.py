"""Known-answer tests for the oracle's MuJoCo restatement.

No MuJoCo exists in this image and the reference holds no physics fixture, so the physics is
"parity unpinned" versus real MuJoCo; these tests pin it to closed-form mechanics instead.
"""
import numpy as np

from oracle import oracle as O

M_TOT = 0.195 + 4 * 0.00693608
HOVER = M_TOT * 9.81 / 4


def _q0(z=1.0):
    return np.array([0, 0, z, 1, 0, 0, 0, 0, 0, 0, 0], float)


def test_k1_free_fall():
    f = O.mj_forward(_q0(), np.zeros(10), np.zeros(4))
    np.testing.assert_allclose(f["qacc"], [0, 0, -9.81, 0, 0, 0, 0, 0, 0, 0], atol=1e-12)
    qp, qv, _, w = O.mj_step(_q0(), np.zeros(10), np.zeros(4))
    assert w == 0
    np.testing.assert_allclose(qv[:3], [0, 0, -0.0981], atol=1e-14)
    np.testing.assert_allclose(qp[:3], [0, 0, 1 - 0.000981], atol=1e-14)  # semi-implicit order


def test_k2_hover_equilibrium():
    f = O.mj_forward(_q0(), np.zeros(10), np.full(4, HOVER))
    np.testing.assert_allclose(f["qacc"], 0, atol=1e-12)


def test_k3_yaw_response():
    d = 0.1
    f = O.mj_forward(_q0(), np.zeros(10), np.array([HOVER + d, HOVER - d, HOVER + d, HOVER - d]))
    tau_z = 4 * d * 0.0201
    izz_eff = 5.37e-4 + 4 * 0.00693608 * 2 * 0.039799 ** 2
    np.testing.assert_allclose(f["qacc"][5], tau_z / izz_eff, rtol=2e-3)
    np.testing.assert_allclose(f["qacc"][6:], -f["qacc"][5], rtol=1e-9)  # props keep spin
    assert abs(f["qacc"][3]) < 1e-6 * abs(f["qacc"][5]) and abs(f["qacc"][4]) < 1e-6 * abs(f["qacc"][5])


def test_k4_linear_drag():
    v = 5.0
    qv = np.zeros(10); qv[0] = v
    f = O.mj_forward(_q0(), qv, np.zeros(4))
    rho, mu = 1.225, 1.8e-5

    def boxes(I, m):
        return [np.sqrt((I[1] + I[2] - I[0]) / m * 6), np.sqrt((I[0] + I[2] - I[1]) / m * 6),
                np.sqrt((I[0] + I[1] - I[2]) / m * 6)]
    bb = boxes([4.16e-4, 4.23e-4, 5.37e-4], 0.195)
    pb = boxes([3.75335e-06, 1.87898e-06, 1.87898e-06], 0.00693608)
    base = 0.5 * rho * bb[1] * bb[2] * v * v + 3 * np.pi * np.mean(bb) * mu * v
    # prop principal axis 1 is -x of the prop frame (inertial quat 0.5 0.5 -0.5 0.5)
    prop = 0.5 * rho * pb[0] * pb[2] * v * v + 3 * np.pi * np.mean(pb) * mu * v
    np.testing.assert_allclose(f["passive"][0], -(base + 4 * prop), rtol=1e-12)
    assert abs(f["passive"][1]) < 1e-15 and abs(f["passive"][2]) < 1e-15


def _com_body():
    mp = 0.00693608
    c = np.array([[0.039799, -0.039799, 0.0336 - 0.001], [-0.039799, -0.039799, 0.032484 + 0.000116422],
                  [-0.039799, 0.039799, 0.033094 - 0.000494174], [0.039799, 0.039799, 0.0336 - 0.001]])
    return mp * c.sum(0) / M_TOT


def _momenta(qp, qv, opt):
    """(angular momentum about the system COM, linear momentum), world frame, via M(q) qdot."""
    h = O.mj_forward(qp, qv, np.zeros(4), opt)["M"] @ qv
    w, x, y, z = qp[3:7] / np.linalg.norm(qp[3:7])
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                  [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                  [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
    P = h[:3]
    return R @ h[3:6] - np.cross(R @ _com_body(), P), P


def test_k5_angular_momentum_conserved_without_fluid():
    opt = O.default_opt(); opt.density = 0.0; opt.viscosity = 0.0
    rng = np.random.default_rng(3)
    qp = _q0(); qv = np.zeros(10)
    qv[0:3] = rng.normal(0, 1, 3); qv[3:6] = rng.normal(0, 3, 3); qv[6:] = rng.normal(0, 20, 4)
    L0, P0 = _momenta(qp, qv, opt)
    for _ in range(100):
        qp, qv, _, _ = O.mj_step(qp, qv, np.zeros(4), opt)
    L1, P1 = _momenta(qp, qv, opt)
    # linear momentum changes only by gravity (to the integrator's first-order error)
    np.testing.assert_allclose(P1[:2], P0[:2], rtol=0, atol=1e-4 * np.linalg.norm(P0))
    np.testing.assert_allclose(P1[2], P0[2] - M_TOT * 9.81 * 1.0, rtol=1e-4)
    # gravity exerts no torque about the COM: L is conserved up to the Euler integrator's error
    assert np.linalg.norm(L1 - L0) < 5e-3 * np.linalg.norm(L0), (L0, L1)
    # first-order convergence: halving dt halves the drift
    opt2 = O.default_opt(); opt2.density = 0.0; opt2.viscosity = 0.0; opt2.timestep = 0.005
    qp2 = _q0(); qv2 = np.zeros(10)
    rng = np.random.default_rng(3)
    qv2[0:3] = rng.normal(0, 1, 3); qv2[3:6] = rng.normal(0, 3, 3); qv2[6:] = rng.normal(0, 20, 4)
    for _ in range(200):
        qp2, qv2, _, _ = O.mj_step(qp2, qv2, np.zeros(4), opt2)
    L2, _ = _momenta(qp2, qv2, opt2)
    r = np.linalg.norm(L2 - L0) / np.linalg.norm(L1 - L0)
    assert 0.35 < r < 0.65, r


def test_k6_mixer_columns():
    env = O.Env()
    env.reset_with(np.array([0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0], np.float32),
                   np.array([0, 0, 1], np.float32))
    out = O.out_to_dict(env.step(np.array([-1 + 2 * (4 * HOVER / 52.0), 0, 0, 0], np.float32)))
    np.testing.assert_allclose(out["motor_commands"], HOVER, rtol=1e-6)
    env.reset_with(np.zeros(12, np.float32) + np.float32([0, 0, 1] + [0] * 9), np.zeros(3, np.float32))
    out = O.out_to_dict(env.step(np.array([1.0, 1.0, 1.0, 1.0], np.float32)))
    assert np.all(out["motor_commands"] >= 0) and np.all(out["motor_commands"] <= 13.0)


def test_bad_ctrl_zeroes_controls():
    qp, qv, ct, w = O.mj_step(_q0(), np.zeros(10), np.array([np.nan, 1, 1, 1]))
    assert w & 4 and np.all(ct == 0)
    np.testing.assert_allclose(qv[2], -0.0981, atol=1e-14)


def test_mass_matrix_spd_and_symmetric():
    rng = np.random.default_rng(0)
    for _ in range(20):
        qp = _q0(); qp[3:7] = rng.normal(size=4); qp[7:] = rng.uniform(-9, 9, 4)
        f = O.mj_forward(qp, rng.normal(size=10), rng.uniform(0, 13, 4))
        M = f["M"]
        assert np.abs(M - M.T).max() == 0
        assert np.linalg.eigvalsh(M).min() > 1e-6
        # mj_solveM agrees with a dense solve
        rhs = f["passive"] + f["actuator"] - f["bias"]
        np.testing.assert_allclose(M @ f["qacc"], rhs, rtol=1e-9, atol=1e-12)


def test_philox_known_answers():
    # Random123 kat_vectors for philox4x32_10
    assert O.philox([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert O.philox([0xffffffff] * 4, [0xffffffff] * 2) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert O.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0]) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_euler_matches_scipy_directly():
    from scipy.spatial.transform import Rotation as R
    rng = np.random.default_rng(5)
    for _ in range(500):
        q = rng.normal(size=4)
        e = O.quat_to_euler(q)
        np.testing.assert_allclose(e, R.from_quat([q[1], q[2], q[3], q[0]]).as_euler("xyz"), atol=1e-13)


def test_brax_oracle_reset_draw_and_free_fall():
    """brax kinds (oracle/brax_oracle.c): reset noise within +-0.01 with the jax_mjx quaternion
    renormalized; from rest at z = 1 with zero motor force (thrust 0, torques 0 -> a = (-1, 0, 0, 0)),
    one step is one semi-implicit Euler step of free fall (drag is zero at rest)."""
    import numpy as np
    from oracle import oracle as O
    for kind in (O.ENV_BRAX_HOVER, O.ENV_BRAX_TRAJ):
        e = O.BraxEnv(kind)
        u = e.draw(3, 17, 0)
        assert np.all(np.abs(u) <= 0.01) and np.unique(u).size == 21
        obs = e.reset_with(u)
        if kind == O.ENV_BRAX_TRAJ:
            assert abs(np.linalg.norm(obs[3:7]) - 1.0) < 1e-6 and abs(obs[2] - 1.0) < 0.011
        else:
            assert np.array_equal(obs[:11], (np.array([0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0], np.float32) + u[:11]))
    e = O.BraxEnv(O.ENV_BRAX_TRAJ)
    obs = e.reset_with(np.zeros(21, np.float32))
    r = e.step(np.array([-1.0, 0.0, 0.0, 0.0], np.float32))
    assert np.allclose(r["motor_commands"], 0.0)
    assert abs(r["obs"][13] - (-9.81 * 0.01)) < 1e-9       # v_z
    assert abs(r["obs"][2] - (1.0 - 9.81 * 0.01 * 0.01)) < 1e-7  # z
    assert not r["terminated"] and not r["truncated"]
