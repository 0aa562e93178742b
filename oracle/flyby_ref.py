"""TEST INFRASTRUCTURE, NOT PRODUCT CODE: scalar restatement of Gameplay/Flyby.cpp:26-196
(Flyby::fly), one statement per reference line, float32 scalars.  Only tests/ use it, as the
checker of gpgpuraytrace_amd/flyby.py (the vectorised product form).

Parity: DirectXMath (XMVector3LengthEst, XMVector3AngleBetweenVectors, XMVectorCatmullRom,
XMVector3Normalize) is absent here, so those are evaluated exactly in float32 -- "parity
unpinned" against the reference binary; the restatement pins the control flow (row `break`,
isnull(score), median rule, turn-around rules) and the arithmetic order.
"""
import math

import numpy as np

f32 = np.float32


def isnull(f):  # Common.h:36-39
    return abs(f32(f)) < f32(0.00001)


def _dot(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def _len(v):
    return f32(math.sqrt(_dot(v, v)))


def _norm(v):
    v = np.asarray(v, np.float32)
    return (v / f32(math.sqrt(_dot(v, v)))).astype(np.float32)


def _angle(a, b):
    c = _dot(a, b) / f32(math.sqrt(_dot(a, a) * _dot(b, b)))
    return f32(math.acos(min(max(float(c), -1.0), 1.0)))


def _catmull(p0, p1, p2, p3, t):
    t = f32(t)
    t2, t3 = t * t, t * t * t
    w0 = (-t3 + f32(2) * t2 - t) * f32(0.5)
    w1 = (f32(3) * t3 - f32(5) * t2 + f32(2)) * f32(0.5)
    w2 = (f32(-3) * t3 + f32(4) * t2 + t) * f32(0.5)
    w3 = (t3 - t2) * f32(0.5)
    return (p0 * w0 + p1 * w1 + p2 * w2 + p3 * w3).astype(np.float32)


class FlybyRef:
    def __init__(self, position, front):
        self.position = np.asarray(position, np.float32)
        self.front = np.asarray(front, np.float32)
        self.reset_target = True
        self.avg_height = f32(0.0)
        self.no_target_time = f32(0.0)
        self.target = np.zeros(3, np.float32)
        self.org = np.zeros(3, np.float32)

    def fly(self, time, view):
        time = f32(time)
        cam_speed = time * f32(4.0)                                        # :28-29
        front, position = self.front, self.position                       # :31-32
        force = np.zeros(3, np.float32)
        score = f32(0.0)
        best = dir_to_best = None
        depth_to_best = f32(0.0)
        view = np.asarray(view, np.float32).reshape(1024, 4)
        for y in range(32):                                                # :40
            for x in range(32):
                cv = view[y * 32 + x]
                vec = cv[:3]
                moved = cv[3]
                if moved < f32(0.0002) or moved > f32(2000.0):            # :46-53
                    break
                strength = moved * moved * moved                           # :56-61
                strength = f32(2.1) - strength
                if strength > f32(0.0):
                    force = (force + (position - vec) * strength * f32(0.0005)).astype(np.float32)
                moved = max(moved - f32(1.5), f32(0.0))                    # :64
                point = f32(0.0)                                           # :67-78
                point += f32(10.0) - abs(moved - f32(10.0))
                hb = cv[1] - self.avg_height
                point += hb * hb
                cs = (16 - abs(x - 16)) + (16 - abs(y - 16))
                point += f32(cs * cs * 2)
                if point > score or isnull(score):                          # :80-87
                    score = point
                    dir_to_best = (vec - position).astype(np.float32)
                    depth_to_best = moved
                    best = (position + dir_to_best * f32(0.3)).astype(np.float32)
        distance = f32(0.0)                                                # :93-104
        if self.reset_target:
            self.reset_target = False
            self.target = (position + np.array([0.1, -0.1, 0.1], np.float32)).astype(np.float32)
            self.avg_height = position[1]
            self.no_target_time = f32(0.0)
        else:
            distance = _len(position - self.target)
        d = sorted(view[:, 3].tolist(), reverse=True)                      # :106-118 nth_element
        median = f32(d[int(f32(1024) * f32(0.2))])
        if f32(0.01) < median < f32(1.4):                                  # :120-127
            distance = f32(0.0)
            score = f32(0.0)
        reached = f32(4.0) * f32(1.2)                                      # :130-131
        if distance < reached:
            if isnull(score):
                self.no_target_time += time
                if self.no_target_time > f32(5.0):
                    self.target = (position - front * f32(2.5)).astype(np.float32)
                    self.no_target_time = f32(0.0)
            else:
                self.no_target_time = f32(0.0)
                self.target = best
                self.org = _norm(dir_to_best)
                if depth_to_best < reached * f32(1.0):
                    if _angle(front, self.target - position) < f32(math.pi / 2):
                        self.target = (position - dir_to_best * f32(2.5)).astype(np.float32)
        dist_to = f32(math.sqrt(_len(self.target - position))) - f32(1.2)  # :171-174
        smooth = max(dist_to * f32(1.8), f32(0.01))
        ang = _angle(front, self.target - position)                        # :176-180
        aim = (f32(2.0) - ang * f32(1.5)) + dist_to * f32(0.1)
        cam_speed = cam_speed * max(min(aim, f32(4.0)), f32(0.1))
        curve = _catmull(position, position + front * smooth, self.target - self.org * smooth * f32(0.2),
                         self.target, time * f32(0.8))                     # :182
        direction = _norm(curve - position)                                # :185-192
        self.front = direction
        force = (force + direction).astype(np.float32)
        self.position = (position + _norm(force) * cam_speed).astype(np.float32)
        sm = f32(1.0) - time * f32(0.1)                                    # :195-196
        self.avg_height = f32(self.avg_height * sm + self.position[1] * (f32(1.0) - sm))
        return self.position, self.front
