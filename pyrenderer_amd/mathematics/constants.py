"""Constants of the hot path (reference: mathematics/constants.py:3-16).

GAMMA_FACTOR is the f32 value Taichi bakes into hit_aabb's
`t_far *= 1 + 2 * GAMMA2_3` (accelerators/bvh_taichi.py:179): 1 + 3*2^-23.
"""
import numpy as np

Pi = 3.14159265358979323846
InvPi = 0.31830988618379067154
Inv2Pi = 0.15915494309189533577
Inv4Pi = 0.07957747154594766788
PiOver2 = 1.57079632679489661923
PiOver4 = 0.78539816339744830961
Sqrt2 = 1.41421356237309504880
finfo = np.finfo(np.float32)
MAX_F = finfo.max
EPS = finfo.tiny
MACHINE_EPS = finfo.eps * 0.5
GAMMA2_3 = (3 * MACHINE_EPS) / (1 - 3 * MACHINE_EPS)
GAMMA_FACTOR = np.float32(1 + 2 * GAMMA2_3)

# core/tracing.py:120 and :127
DIRECT_LIGHT_RGB = (0.9, 0.85, 0.7)
T_MIN = np.float32(0.00001)
T_MAX = np.float32(99999.9)
