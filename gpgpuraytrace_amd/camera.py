"""Camera and frame constants (host side): Graphics/Camera.cpp and the
Terrain/Raytracer code that feeds the shader constants.

The reference uses DirectXMath (absent here); the formulas below restate
XMQuaternionRotationRollPitchYaw, XMVector3Rotate, XMMatrixLookToLH,
XMMatrixPerspectiveFovLH and XMMatrixInverse in float64 and round to float32
(tolerance-level agreement with DirectXMath, documented in DESIGN.md).
"""
import math

import numpy as np

INITIAL_POSITION = (0.0, 100.0, 0.0)        # Camera.cpp:9
INITIAL_ROTATION_EULER = (-3.0, -4.6, 0.0)  # Camera.cpp:10
LOOKDOWN_ROTATION_EULER = (-3.6, -4.6, 0.0)  # build's hit-heavy second pose
FOV_DEG = 80.0                              # Camera.cpp:39
NEAR_Z, FAR_Z = 0.01, 5000.0                # Camera.cpp:19-20
UP = (0.0, -1.0, 0.0)                       # Camera.h:9 XM_UP
FRONT = (0.0, 0.0, 1.0)                     # Camera.h:10 XM_FRONT
XM_2PI = 6.283185307


def quaternion_roll_pitch_yaw(pitch, yaw, roll):
    sp, cp = math.sin(pitch * 0.5), math.cos(pitch * 0.5)
    sy, cy = math.sin(yaw * 0.5), math.cos(yaw * 0.5)
    sr, cr = math.sin(roll * 0.5), math.cos(roll * 0.5)
    return np.array([sp * cy * cr + cp * sy * sr, cp * sy * cr - sp * cy * sr,
                     cp * cy * sr - sp * sy * cr, cp * cy * cr + sp * sy * sr])


def _qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def rotate(v, q):
    conj = np.array([-q[0], -q[1], -q[2], q[3]])
    return _qmul(_qmul(q, np.array([v[0], v[1], v[2], 0.0])), conj)[:3]


def look_to_lh(eye, direction, up):
    r2 = np.asarray(direction, float)
    r2 = r2 / np.linalg.norm(r2)
    r0 = np.cross(up, r2)
    r0 = r0 / np.linalg.norm(r0)
    r1 = np.cross(r2, r0)
    ne = -np.asarray(eye, float)
    m = np.zeros((4, 4))
    m[0:3, 0], m[0:3, 1], m[0:3, 2] = r0, r1, r2
    m[3, 0:3] = [r0 @ ne, r1 @ ne, r2 @ ne]
    m[3, 3] = 1.0
    return m


def perspective_fov_lh(fov, aspect, zn, zf):
    h = math.cos(0.5 * fov) / math.sin(0.5 * fov)
    r = zf / (zf - zn)
    m = np.zeros((4, 4))
    m[0, 0], m[1, 1], m[2, 2], m[2, 3], m[3, 2] = h / aspect, h, r, 1.0, -r * zn
    return m


class Camera:
    """Camera.cpp: position + euler rotation -> View / Projection matrices."""

    def __init__(self, width, height, position=INITIAL_POSITION, euler=INITIAL_ROTATION_EULER):
        self.width, self.height = int(width), int(height)
        self.position = np.array(position, float)
        self.rotation_euler = list(euler)
        aspect = float(np.float32(self.width) / np.float32(self.height))
        self.mat_projection = perspective_fov_lh(math.radians(FOV_DEG), aspect, NEAR_Z, FAR_Z)  # Camera.cpp:39-42
        self.rotate()
        self.update()

    def rotate(self):  # Camera.cpp:101-106
        q = quaternion_roll_pitch_yaw(self.rotation_euler[0], self.rotation_euler[1], 0.0)
        self.front = rotate(FRONT, q)

    def update(self):  # Camera.cpp:108-113
        self.mat_view = look_to_lh(self.position, self.front, np.array(UP))

    # --- what Terrain writes into the shaders ---
    def view_inverse_hlsl(self):
        """ViewInverse as the shader sees it (Terrain.cpp:305: transpose(inverse(View)) uploaded,
        column_major packing turns it back into inverse(View))."""
        return np.linalg.inv(self.mat_view).astype(np.float32)

    def projection_hlsl(self):
        return self.mat_projection.astype(np.float32)

    def eye(self):
        return np.array([self.position[0], self.position[1], self.position[2], 0.0], np.float32)


def sun_direction(time_of_day):
    """Terrain::setTimeOfDay (Terrain.cpp:285-300)."""
    s = np.array([-math.sin(time_of_day * XM_2PI), -math.cos(time_of_day * XM_2PI), 0.1])
    return (s / np.linalg.norm(s)).astype(np.float32)


def cbuffer_bytes_matrix(m_hlsl):
    """Bytes the engine writes for a float4x4 variable: the row-major bytes of transpose(M)."""
    return np.ascontiguousarray(np.asarray(m_hlsl, np.float32).T).tobytes()


def camera_constants(cam, time_of_day=0.3):
    """The shader constants of a camera's current state (after Camera.update)."""
    return {"width": cam.width, "height": cam.height, "eye": cam.eye(),
            "view_inverse": cam.view_inverse_hlsl(), "projection": cam.projection_hlsl(),
            "sun": sun_direction(time_of_day)}


def frame_constants(width, height, position=INITIAL_POSITION, euler=INITIAL_ROTATION_EULER, time_of_day=0.3):
    return camera_constants(Camera(width, height, position, euler), time_of_day)
