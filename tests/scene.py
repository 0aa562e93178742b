"""Frame constants for the fixed benchmark scene (TEST INFRASTRUCTURE).

A numpy float32 restatement of the DirectXMath calls the reference makes
(Camera.cpp:9-10,39-42,101-113; Terrain.cpp:285-311); DirectXMath is not in
this image, so these are tolerance-level (parity unpinned) -- kernel parity
never depends on them because the fixtures carry the matrices themselves.
"""
import math

import numpy as np

f32 = np.float32
RESET_EYE = (0.0, 100.0, 0.0)
RESET_EULER = (-3.0, -4.6, 0.0)      # Camera.cpp:10
LOOKDOWN_EULER = (-3.6, -4.6, 0.0)   # build's second, hit-heavy pose
TIME_OF_DAY = 0.3                    # Raytracer.cpp:31


def _quat_rpy(pitch, yaw, roll):
    # XMQuaternionRotationRollPitchYaw
    sp, cp = math.sin(pitch * 0.5), math.cos(pitch * 0.5)
    sy, cy = math.sin(yaw * 0.5), math.cos(yaw * 0.5)
    sr, cr = math.sin(roll * 0.5), math.cos(roll * 0.5)
    return np.array([sp * cy * cr + cp * sy * sr, cp * sy * cr - sp * cy * sr,
                     cp * cy * sr - sp * sy * cr, cp * cy * cr + sp * sy * sr], np.float64)


def _qmul(a, b):  # Hamilton product a*b, (x,y,z,w)
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def _rotate(v, q):  # XMVector3Rotate: q * v * conj(q)
    conj = np.array([-q[0], -q[1], -q[2], q[3]])
    return _qmul(_qmul(q, np.array([v[0], v[1], v[2], 0.0])), conj)[:3]


def look_to_lh(eye, front, up):
    # XMMatrixLookToLH (row-vector convention)
    r2 = front / np.linalg.norm(front)
    r0 = np.cross(up, r2)
    r0 = r0 / np.linalg.norm(r0)
    r1 = np.cross(r2, r0)
    ne = -np.asarray(eye, np.float64)
    m = np.zeros((4, 4))
    m[0:3, 0] = r0
    m[0:3, 1] = r1
    m[0:3, 2] = r2
    m[3, 0:3] = [r0 @ ne, r1 @ ne, r2 @ ne]
    m[3, 3] = 1.0
    return m


def perspective_fov_lh(fov, aspect, zn, zf):
    # XMMatrixPerspectiveFovLH
    h = math.cos(0.5 * fov) / math.sin(0.5 * fov)
    w = h / aspect
    r = zf / (zf - zn)
    m = np.zeros((4, 4))
    m[0, 0], m[1, 1], m[2, 2], m[2, 3], m[3, 2] = w, h, r, 1.0, -r * zn
    return m


def frame_constants(width, height, eye=RESET_EYE, euler=RESET_EULER, time_of_day=TIME_OF_DAY):
    q = _quat_rpy(euler[0], euler[1], euler[2])
    front = _rotate((0.0, 0.0, 1.0), q)
    view = look_to_lh(np.asarray(eye, np.float64), front, np.array([0.0, -1.0, 0.0]))
    proj = perspective_fov_lh(math.radians(80.0), float(f32(width) / f32(height)), 0.01, 5000.0)
    vinv = np.linalg.inv(view)
    two_pi = 6.283185307
    sun = np.array([-math.sin(time_of_day * two_pi), -math.cos(time_of_day * two_pi), 0.1])
    sun = sun / np.linalg.norm(sun)
    return {
        "width": int(width), "height": int(height),
        "eye": np.array([eye[0], eye[1], eye[2], 0.0], np.float32),
        "view_inverse": vinv.astype(np.float32),     # HLSL ViewInverse (= inverse(View))
        "projection": proj.astype(np.float32),       # HLSL Projection
        "sun": sun.astype(np.float32),
    }
