"""Minimal stand-in for the mujoco bindings (golden-vector generation only).

mj_step delegates to the CPU oracle's restatement of MuJoCo's Euler step for drone.xml.
"""
import numpy as np

STEP_FN = None  # injected by tools/gen_golden.py: f(qpos, qvel, ctrl) in place


class _Opt:
    timestep = 0.01


class MjModel:
    nq, nv, nu = 11, 10, 4
    qpos0 = np.array([0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0], dtype=np.float64)

    def __init__(self):
        self.opt = _Opt()

    @staticmethod
    def from_xml_path(path):
        return MjModel()


class MjData:
    def __init__(self, m):
        self.qpos = m.qpos0.copy()
        self.qvel = np.zeros(m.nv)
        self.ctrl = np.zeros(m.nu)


def mj_resetData(m, d):
    d.qpos[:] = m.qpos0
    d.qvel[:] = 0
    d.ctrl[:] = 0


def mj_forward(m, d):
    pass


def mj_step(m, d):
    STEP_FN(d.qpos, d.qvel, d.ctrl)
