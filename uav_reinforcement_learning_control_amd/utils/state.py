"""QuadState with the reference's interface (utils/state.py:9-108): the 12-D state
[x, y, z, roll, pitch, yaw, vx, vy, vz, wx, wy, wz] as float32, with conversions to and from
MuJoCo's qpos / qvel (quaternion w x y z).

The attitude conversions are the ones scipy's Rotation performs for the 'xyz' (extrinsic) sequence
the reference uses: quaternion -> Euler by Bernardes & Viollet's method (scipy's algorithm,
including its gimbal-lock branch), Euler -> quaternion as q = qz(yaw) qy(pitch) qx(roll). They are
computed here in float64 numpy (scipy is not needed); the step kernels compute the same in float32
(csrc/quad_physics.h quat_to_euler / euler_to_quat). Matches the reference's float32 state bit for
bit on tests/golden/golden_euler.npz.
"""
from __future__ import annotations

import numpy as np

_PI = np.pi


def quat_to_euler_xyz(q_wxyz) -> np.ndarray:
    """Rotation.from_quat(xyzw).as_euler('xyz') for a (not necessarily unit) wxyz quaternion."""
    q = np.asarray(q_wxyz, np.float64)
    q = q / np.sqrt(np.dot(q, q))
    w, x, y, z = q
    # extrinsic xyz == intrinsic ZYX reversed: Bernardes & Viollet with (i, j, k) = (2, 1, 0)
    # and the sign for the odd permutation
    a, b, c, d = w - y, x + z, y + w, z - x
    mid = 2.0 * np.arctan2(np.hypot(c, d), np.hypot(a, b))
    hs, hd = np.arctan2(b, a), np.arctan2(d, c)
    eps = 1e-7
    if abs(mid) <= eps:
        e = np.array([2.0 * hs, mid, 0.0])
    elif abs(mid - _PI) <= eps:
        e = np.array([-2.0 * hd, mid, 0.0])
    else:
        e = np.array([hs - hd, mid, hs + hd])
    e[1] -= _PI / 2.0
    return np.where(e < -_PI, e + 2 * _PI, np.where(e > _PI, e - 2 * _PI, e))


def euler_xyz_to_quat(e) -> np.ndarray:
    """Rotation.from_euler('xyz', e).as_quat() as w x y z: the extrinsic composition
    q = qz(yaw) (qy(pitch) qx(roll)), built one elementary rotation at a time (no w >= 0 flip)."""
    h = 0.5 * np.asarray(e, np.float64)
    v, w = np.array([np.sin(h[0]), 0.0, 0.0]), np.cos(h[0])
    for ax in (1, 2):
        pv = np.zeros(3)
        pv[ax], pw = np.sin(h[ax]), np.cos(h[ax])
        v, w = pw * v + w * pv + np.cross(pv, v), pw * w - np.dot(pv, v)
    return np.array([w, v[0], v[1], v[2]])


class QuadState:
    """12-D quadrotor state: position, roll/pitch/yaw (rad), world velocity, body rates."""

    ROT_SEQ = "XYZ"

    def __init__(self, obs_bounds=None):
        self.state = np.zeros(12, dtype=np.float32)
        self.obs_bounds = obs_bounds

    def set_from_mujoco(self, qpos: np.ndarray, qvel: np.ndarray) -> None:
        """qpos [x y z qw qx qy qz ...], qvel [vx vy vz wx wy wz ...]."""
        self.state[0:3] = qpos[0:3]
        self.state[3:6] = quat_to_euler_xyz(qpos[3:7])
        self.state[6:9] = qvel[0:3]
        self.state[9:12] = qvel[3:6]

    def get_mujoco_state(self) -> tuple[np.ndarray, np.ndarray]:
        """(qpos[7], qvel[6]) for MuJoCo from the current state."""
        qpos = np.concatenate([self.state[0:3], euler_xyz_to_quat(self.state[3:6])])
        return qpos, self.state[6:12].copy()

    def reset_uav_state(self, pos: np.ndarray, wxyz: np.ndarray, vel: np.ndarray, ang_vel: np.ndarray):
        self.state[0:3] = pos
        self.state[3:6] = quat_to_euler_xyz(np.asarray(wxyz, np.float64))
        self.state[6:9] = vel
        self.state[9:12] = ang_vel

    @property
    def position(self) -> np.ndarray:
        return self.state[0:3]

    @property
    def attitude(self) -> np.ndarray:
        return self.state[3:6]

    @property
    def velocity(self) -> np.ndarray:
        return self.state[6:9]

    @property
    def angular_velocity(self) -> np.ndarray:
        return self.state[9:12]

    def random_reset(self, rng: np.random.Generator, bounds) -> None:
        """Uniform draw within bounds.low / bounds.high (12 float64 draws, stored as float32)."""
        self.state = rng.uniform(bounds.low, bounds.high).astype(np.float32)

    def vec(self) -> np.ndarray:
        return self.state.copy()

    def __repr__(self) -> str:
        return (f"QuadState(pos={self.position}, att={np.rad2deg(self.attitude)}, "
                f"vel={self.velocity}, ang_vel={self.angular_velocity})")
