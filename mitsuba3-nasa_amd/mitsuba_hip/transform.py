"""ScalarTransform4f restated on numpy (float64 internally, float32 on export).

Mirrors include/mitsuba/core/transform.h (translate / scale / rotate /
look_at / perspective and composition) and the Dr.Jit matrix helpers it
calls.  The reference evaluates these in float32; evaluating in float64 and
rounding once changes scene constants by at most an ulp.
"""
from __future__ import annotations

import math

import numpy as np


class _chain:
    """``T.translate(v)`` builds a transform; ``t.translate(v)`` composes
    ``t @ translate(v)`` — the ChainTransform4f binding of the reference
    (src/core/python/transform_v.cpp:136-214)."""

    def __init__(self, builder):
        self.builder = builder

    def __get__(self, obj, cls):
        if obj is None:
            return lambda *a, **k: self.builder(*a, **k)
        return lambda *a, **k: obj @ self.builder(*a, **k)


class Transform4f:
    __slots__ = ("matrix", "inverse_transpose")

    def __init__(self, matrix=None, inverse_transpose=None):
        m = np.eye(4) if matrix is None else np.array(matrix, dtype=np.float64).reshape(4, 4)
        self.matrix = m
        self.inverse_transpose = (np.linalg.inv(m).T if inverse_transpose is None
                                  else np.array(inverse_transpose, dtype=np.float64))

    # -- composition (transform.h:66-69) --------------------------------------
    def __matmul__(self, other):
        if isinstance(other, Transform4f):
            return Transform4f(self.matrix @ other.matrix,
                               self.inverse_transpose @ other.inverse_transpose)
        return self.transform_point(other)

    __mul__ = __matmul__

    def inverse(self):
        return Transform4f(self.inverse_transpose.T, self.matrix.T)

    @staticmethod
    def Translate(v):
        v = np.broadcast_to(np.asarray(v, dtype=np.float64), (3,))
        m = np.eye(4)
        m[:3, 3] = v
        mi = np.eye(4)
        mi[:3, 3] = -v
        return Transform4f(m, mi.T)

    @staticmethod
    def Scale(v):
        v = np.broadcast_to(np.asarray(v, dtype=np.float64), (3,))
        m = np.diag([v[0], v[1], v[2], 1.0])
        mi = np.diag([1.0 / v[0], 1.0 / v[1], 1.0 / v[2], 1.0])
        return Transform4f(m, mi)

    @staticmethod
    def Rotate(axis, angle_deg):
        # dr::rotate<Matrix4f>(axis, deg_to_rad(angle)) — Rodrigues form
        a = np.asarray(axis, dtype=np.float64)
        a = a / np.linalg.norm(a)
        th = math.radians(angle_deg)
        s, c = math.sin(th), math.cos(th)
        t = 1.0 - c
        x, y, z = a
        r = np.array([[x * x * t + c, x * y * t - z * s, x * z * t + y * s, 0],
                      [x * y * t + z * s, y * y * t + c, y * z * t - x * s, 0],
                      [x * z * t - y * s, y * z * t + x * s, z * z * t + c, 0],
                      [0, 0, 0, 1]])
        return Transform4f(r, r)

    @staticmethod
    def LookAt(origin, target, up):
        # transform.h:254-283
        o = np.asarray(origin, dtype=np.float64)
        d = np.asarray(target, dtype=np.float64) - o
        d /= np.linalg.norm(d)
        left = np.cross(np.asarray(up, dtype=np.float64), d)
        left /= np.linalg.norm(left)
        new_up = np.cross(d, left)
        m = np.eye(4)
        m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = left, new_up, d, o
        return Transform4f(m)

    @staticmethod
    def Perspective(fov, near, far):
        # transform.h:215-233
        recip = 1.0 / (far - near)
        tan = math.tan(math.radians(fov * 0.5))
        cot = 1.0 / tan
        m = np.diag([cot, cot, far * recip, 0.0])
        m[2, 3] = -near * far * recip
        m[3, 2] = 1.0
        return Transform4f(m)

    # -- application ------------------------------------------------------------
    def transform_point(self, p):
        p = np.asarray(p, dtype=np.float64)
        r = self.matrix @ np.append(p, 1.0)
        return r[:3] / r[3]

    def transform_vector(self, v):
        return self.matrix[:3, :3] @ np.asarray(v, dtype=np.float64)

    def transform_normal(self, n):
        return self.inverse_transpose[:3, :3] @ np.asarray(n, dtype=np.float64)

    def has_scale(self):
        m = self.matrix[:3, :3]
        return not np.allclose(np.linalg.norm(m, axis=0), 1.0, atol=1e-3)

    def __repr__(self):
        return f"Transform4f({self.matrix.tolist()})"


Transform4f.translate = _chain(Transform4f.Translate)
Transform4f.scale = _chain(Transform4f.Scale)
Transform4f.rotate = _chain(Transform4f.Rotate)
Transform4f.look_at = _chain(Transform4f.LookAt)
Transform4f.perspective = _chain(Transform4f.Perspective)

ScalarTransform4f = Transform4f
