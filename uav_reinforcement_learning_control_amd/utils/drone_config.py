"""Physical constants of the reference drone (utils/drone_config.py:9-22 of the reference).
The HIP kernels take these through QuadCfg (include/quadenv.h); this module is for callers."""
MAX_MOTOR_THRUST = 13.0
ARM_LENGTH = 0.039799
YAW_TORQUE_COEFF = 0.0201
MASS = 0.2227
G = 9.81
DT = 0.01
IXX = 4.16e-4
IYY = 4.23e-4
IZZ = 5.37e-4
MAX_TOTAL_THRUST = 4 * MAX_MOTOR_THRUST
MAX_TORQUE = 0.5
HOVER_THRUST_PER_MOTOR = MASS * G / 4
