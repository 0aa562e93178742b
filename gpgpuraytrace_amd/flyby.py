"""Flyby autopilot: Gameplay/Flyby.cpp:26-196, the only other consumer of
the camerarays prepass.  Each frame it scores the 32x32 CameraResults of the previous frame
(Terrain::getCameraView), picks a target, and steers the camera along a Catmull-Rom curve.

Host code over numpy float32 (the reference's XMVECTOR lanes are float32).  The point scan is
vectorised: per-row validity (the `break` on an unusable depth, :44-50), the collision force
accumulated in scan order (np.add.accumulate: the same sequential float32 sums), and the best
point as a strict running maximum that starts at the first usable point (:80, the isnull(score)
rule); a running score that is itself ~0 (where isnull lets a lower point replace it) drops to
the scalar scan.  DirectXMath's estimate functions (XMVector3LengthEst, XMVectorACos inside
XMVector3AngleBetweenVectors) are evaluated exactly: DirectXMath is not available here, so paths
are pinned to tests/'s scalar restatement (oracle/flyby_ref.py), not to the reference binary.
std::nth_element's reordering of the view (:110-117) is not reproduced (its order is unspecified);
only the selected depth is used.
"""
import math

import numpy as np

from .camera import Camera

RES = 32
CAM_SPEED_MULT = np.float32(4.0)
POINT_REACHED = np.float32(CAM_SPEED_MULT * np.float32(1.2))
f32 = np.float32


def _dot(a, b):
    """XMVector3Dot in a fixed float32 order ((x*x + y*y) + z*z), no BLAS reduction."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2])


def _norm(v):
    v = np.asarray(v, np.float32)
    return (v / f32(np.sqrt(_dot(v, v)))).astype(np.float32)


def _length(v):
    return f32(np.sqrt(_dot(v, v)))


def _angle(a, b):
    """XMVector3AngleBetweenVectors: acos(clamp(dot(a, b) / (|a| |b|), -1, 1))."""
    c = _dot(a, b) / f32(np.sqrt(_dot(a, a) * _dot(b, b)))
    return f32(math.acos(min(max(float(c), -1.0), 1.0)))  # acos in double, rounded once


def catmull_rom(p0, p1, p2, p3, t):
    """XMVectorCatmullRom."""
    t = f32(t)
    t2, t3 = t * t, t * t * t
    w0 = (-t3 + f32(2) * t2 - t) * f32(0.5)
    w1 = (f32(3) * t3 - f32(5) * t2 + f32(2)) * f32(0.5)
    w2 = (f32(-3) * t3 + f32(4) * t2 + t) * f32(0.5)
    w3 = (t3 - t2) * f32(0.5)
    return (p0 * w0 + p1 * w1 + p2 * w2 + p3 * w3).astype(np.float32)


class Flyby:
    """Gameplay/Flyby.{h,cpp}.  `camera` is a camera.Camera (position / front are read and
    written, as Flyby does with Camera's public members)."""

    def __init__(self, camera: Camera):
        self.camera = camera
        self.reset_target = True  # Flyby.cpp:9-14
        self.avg_height = f32(0.0)
        self.no_target_time = f32(0.0)
        self.target = np.zeros(3, np.float32)
        self.org_dir_to_target = np.zeros(3, np.float32)  # uninitialised in the reference until a target is set
        self.log = []  # Logger() lines of the last fly()

    def reset(self):  # Flyby.cpp:21-24
        self.reset_target = True

    def _scan(self, view, position):
        d = view[:, 3].reshape(RES, RES)
        bad = (d < f32(0.0002)) | (d > f32(2000.0))
        first_bad = np.where(bad.any(1), bad.argmax(1), RES)
        valid = (np.arange(RES)[None, :] < first_bad[:, None]).ravel()
        idx = np.nonzero(valid)[0]
        force = np.zeros(3, np.float32)
        if idx.size == 0:
            return force, f32(0.0), None
        v = view[idx]
        vec, depth = v[:, :3], v[:, 3]
        strength = f32(2.1) - depth * depth * depth
        push = (position[None, :] - vec) * strength[:, None] * f32(0.0005)
        push = push[strength > f32(0.0)]
        if len(push):
            force = np.add.accumulate(np.vstack([np.zeros((1, 3), np.float32), push]), axis=0,
                                      dtype=np.float32)[-1]
        moved = np.maximum(depth - f32(1.5), f32(0.0))
        score = f32(10.0) - np.abs(moved - f32(10.0))
        hb = v[:, 1] - self.avg_height
        score = score + hb * hb
        x, y = idx % RES, idx // RES
        cs = (RES // 2 - np.abs(x - RES // 2)) + (RES // 2 - np.abs(y - RES // 2))
        score = (score + (cs * cs * 2).astype(np.float32)).astype(np.float32)
        # strict running maximum from the first usable point (Flyby.cpp:80)
        run = np.maximum.accumulate(score)
        if np.any(np.abs(run) < f32(0.00001)):
            best_i, best = 0, score[0]
            for i in range(1, len(score)):
                if score[i] > best or abs(best) < 0.00001:
                    best_i, best = i, score[i]
        else:
            best = run[-1]
            best_i = int(np.argmax(score == best))
        return force, f32(best), (vec[best_i], moved[best_i])

    def fly(self, time, view):
        """Flyby::fly(time, terrain): `view` = the (1024, 4) CameraResults of the previous frame."""
        cam = self.camera
        time = f32(time)
        self.log = []
        cam_speed = time * CAM_SPEED_MULT
        front = np.asarray(cam.front, np.float32)
        position = np.asarray(cam.position, np.float32)
        view = np.asarray(view, np.float32).reshape(RES * RES, 4)
        force, score, pick = self._scan(view, position)
        if pick is not None:
            dir_to_best = (pick[0] - position).astype(np.float32)
            depth_to_best = pick[1]
            best = (position + dir_to_best * f32(0.3)).astype(np.float32)
        distance = f32(0.0)
        if self.reset_target:  # :93-104
            self.reset_target = False
            self.target = (position + np.array([0.1, -0.1, 0.1], np.float32)).astype(np.float32)
            self.avg_height = position[1]
            self.no_target_time = f32(0.0)
        else:
            distance = _length(position - self.target)
        # 20% "median": the element nth_element puts at index size*0.2 with depth descending (:106-118)
        depths = view[:, 3]
        median = f32(np.sort(depths)[::-1][int(np.float32(len(depths)) * np.float32(0.2))])
        if f32(0.01) < median < f32(1.4):  # :120-127
            distance = f32(0.0)
            score = f32(0.0)
            self.log.append(f"Median depth is {median} so assuming our current direction is impossible")
        if distance < POINT_REACHED:  # :130-166
            if abs(score) < 0.00001:
                self.log.append("No new target found")
                self.no_target_time += time
                if self.no_target_time > f32(5.0):
                    self.target = (position - front * f32(2.5)).astype(np.float32)
                    self.log.append("Turning around cause of no target")
                    self.no_target_time = f32(0.0)
            else:
                self.no_target_time = f32(0.0)
                self.log.append(f"Setting new target with score {score}")
                self.target = best
                self.org_dir_to_target = _norm(dir_to_best)
                if depth_to_best < POINT_REACHED * f32(1.0):
                    angle = _angle(front, self.target - position)
                    if angle < f32(np.pi / 2):
                        self.target = (position - dir_to_best * f32(2.5)).astype(np.float32)
                        self.log.append("Turning around because point is too close")
        # next position on the curve (:168-192)
        dist_to_target = f32(np.sqrt(_length(self.target - position))) - f32(1.2)
        smooth = max(dist_to_target * f32(1.8), f32(0.01))
        angle_to_target = _angle(front, self.target - position)
        aim = (f32(2.0) - angle_to_target * f32(1.5)) + dist_to_target * f32(0.1)
        cam_speed = cam_speed * max(min(aim, f32(4.0)), f32(0.1))
        curve = catmull_rom(position, position + front * smooth,
                            self.target - self.org_dir_to_target * smooth * f32(0.2), self.target, time * f32(0.8))
        direction = _norm(curve - position)
        cam.front = direction.astype(np.float64)
        force = (force + direction).astype(np.float32)
        cam.position = (position + _norm(force) * cam_speed).astype(np.float64)
        smoother = f32(1.0) - time * f32(0.1)
        self.avg_height = f32(self.avg_height * smoother + f32(cam.position[1]) * (f32(1.0) - smoother))
        return cam


def fly_through(ring_or_terrain, camera, frames, dt=1.0 / 25.0, recorder=None, shard=(0, 1)):
    """The reference's fixed-frame-rate fly-through (Raytracer.cpp:116-121 record mode, :141
    1/TARGET_FRAME_RATE steps; loop :129-192): per frame Flyby::fly on the previous frame's
    camera view, Camera::update, then render + present.  Works on a Terrain or an
    engine.FrameRing (frames in flight: frame i+1 is set up as soon as frame i's prepass
    results arrive, while frame i's tracescreen still runs).  Returns the camera path,
    (frames, 2, 3) float64 positions and fronts."""
    from .engine import FrameRing
    ring = ring_or_terrain if isinstance(ring_or_terrain, FrameRing) else None
    fly = Flyby(camera)
    fly.reset()
    view = np.zeros((RES * RES, 4), np.float32)  # Terrain's zero-initialised cameraView on frame 1
    path = []
    for _ in range(frames):
        fly.fly(dt, view)
        camera.update()
        path.append((camera.position.copy(), np.asarray(camera.front, float).copy()))
        if ring is not None:
            dev, ter = ring.next_slot()
            ter.set_camera(camera)
            ter.update_terrain()
            ter.render_device(shard[0], shard[1], feed=True)
            ring.frame += 1
        else:
            ter = ring_or_terrain
            dev = ter.device
            ter.set_camera(camera)
            ter.update_terrain()
            ter.render_device(shard[0], shard[1], feed=True)
        if recorder is not None:
            recorder.set_frame_time(dt)
        dev.present()
        view = ter.camera_feed().copy()
    return np.array(path)
