"""mi.load_file / mi.load_string for the hot path's plugins (SURVEY.md §8(f)
rank 2; src/core/xml.cpp).

Parses the Mitsuba 3 scene XML into the dictionary form that `load_dict`
takes: `<default>` and `$name` substitution, `<integer|float|boolean|string|
rgb|spectrum|point|vector>` properties, `<transform>` chains (translate,
rotate, scale, matrix, lookat; each applied after the previous one as in
xml.cpp), nested objects (bsdf, texture, emitter, medium, phase, volume,
sampler, film, rfilter), `<ref>` and relative file names resolved against the
file's directory.  Objects keep their `id` as the dictionary key (so
`mi.traverse` keys match the reference's); unnamed ones get `_unnamed_<n>`.
"""
from __future__ import annotations

import os
import re
import xml.etree.ElementTree as ET
from typing import Any, Dict

import numpy as np

from .transform import Transform4f

_OBJECT_TAGS = {"scene", "integrator", "sensor", "bsdf", "texture", "emitter", "shape", "medium", "phase",
                "volume", "sampler", "film", "rfilter"}
# property name of a nested object without a name attribute
_DEFAULT_SLOT = {"bsdf": "bsdf", "emitter": "emitter", "sampler": "sampler", "film": "film",
                 "rfilter": "rfilter", "phase": "phase", "medium": "medium"}
_FILE_KEYS = {"filename"}


def _subst(s: str, params: Dict[str, str]) -> str:
    def rep(m):
        k = m.group(1)
        if k not in params:
            raise RuntimeError(f'xml: undefined parameter "${k}"')
        return str(params[k])
    return re.sub(r"\$([A-Za-z_][A-Za-z0-9_]*)", rep, s)


def _floats(s: str):
    return [float(x) for x in re.split(r"[,\s]+", s.strip()) if x]


def _vec3(el, params, default=0.0):
    if "value" in el.attrib:
        v = _floats(_subst(el.attrib["value"], params))
        return v * 3 if len(v) == 1 else v
    return [float(_subst(el.attrib.get(k, str(default)), params)) for k in ("x", "y", "z")]


def _transform(el, params) -> Transform4f:
    T = Transform4f()
    for op in el:
        tag = op.tag
        if tag == "translate":
            M = Transform4f.translate(_vec3(op, params))
        elif tag == "scale":
            if "value" in op.attrib:
                v = _floats(_subst(op.attrib["value"], params))
                v = v * 3 if len(v) == 1 else v
            else:
                v = [float(_subst(op.attrib.get(k, "1"), params)) for k in ("x", "y", "z")]
            M = Transform4f.scale(v)
        elif tag == "rotate":
            axis = _vec3(op, params)
            M = Transform4f.rotate(axis, float(_subst(op.attrib["angle"], params)))
        elif tag == "matrix":
            v = _floats(_subst(op.attrib["value"], params))
            if len(v) == 9:
                m = np.eye(4)
                m[:3, :3] = np.asarray(v).reshape(3, 3)
            elif len(v) == 16:
                m = np.asarray(v).reshape(4, 4)
            else:
                raise RuntimeError("xml: <matrix> expects 9 or 16 values")
            M = Transform4f(m)
        elif tag == "lookat":
            g = lambda k: _floats(_subst(op.attrib[k], params))
            M = Transform4f.look_at(origin=g("origin"), target=g("target"),
                                    up=g("up") if "up" in op.attrib else [0, 1, 0])
        else:
            raise RuntimeError(f'xml: unsupported transform operation <{tag}>')
        T = M @ T
    return T


class _Parser:
    def __init__(self, base_dir: str, params: Dict[str, Any]):
        self.base_dir = base_dir
        self.params = {k: str(v) for k, v in params.items()}
        self.unnamed = 0

    def value(self, el):
        tag, p = el.tag, self.params
        raw = _subst(el.attrib.get("value", ""), p)
        if tag == "integer":
            return int(raw)
        if tag == "float":
            return float(raw)
        if tag == "boolean":
            return raw.strip().lower() == "true"
        if tag == "string":
            if el.attrib.get("name") in _FILE_KEYS and raw and not os.path.isabs(raw):
                return os.path.join(self.base_dir, raw)
            return raw
        if tag in ("rgb", "spectrum"):
            v = _floats(raw)
            return {"type": "rgb", "value": v * 3 if len(v) == 1 else v}
        if tag in ("point", "vector"):
            return _vec3(el, p)
        if tag == "transform":
            return _transform(el, p)
        raise RuntimeError(f"xml: unsupported property <{tag}>")

    def obj(self, el) -> Dict[str, Any]:
        d: Dict[str, Any] = {"type": _subst(el.attrib["type"], self.params)} if "type" in el.attrib else {}
        for c in el:
            if c.tag == "default":
                self.params.setdefault(c.attrib["name"], _subst(c.attrib["value"], self.params))
                continue
            name = c.attrib.get("name")
            if c.tag == "ref":
                d[name or "bsdf"] = {"type": "ref", "id": _subst(c.attrib["id"], self.params)}
            elif c.tag in _OBJECT_TAGS:
                sub = self.obj(c)
                if el.tag == "scene":
                    key = c.attrib.get("id") or (c.tag if c.tag in ("integrator", "sensor") else None)
                else:
                    key = name or _DEFAULT_SLOT.get(c.tag) or c.attrib.get("id")
                if key is None:
                    key = f"_unnamed_{self.unnamed}"
                    self.unnamed += 1
                if key in d:
                    raise RuntimeError(f'xml: duplicate object or property "{key}"')
                d[key] = sub
            elif c.tag == "include":
                raise RuntimeError("xml: <include> is not supported by the hip_ad_rgb loader")
            else:
                d[name] = self.value(c)
        return d


def load_string(s: str, base_dir: str = ".", **params):
    """mi.load_string: returns what load_dict returns for the parsed scene."""
    from .scene import load_dict
    root = ET.fromstring(s)
    if root.tag != "scene":
        raise RuntimeError(f'xml: root element must be <scene>, got <{root.tag}>')
    ver = root.attrib.get("version", "3.0.0")
    if not ver.startswith(("2.", "3.")):
        raise RuntimeError(f"xml: unsupported scene version {ver}")
    d = _Parser(base_dir, params).obj(root)
    d["type"] = "scene"
    return load_dict(d)


def load_file(path: str, **params):
    """mi.load_file (core/xml.cpp:load_file) with `$name` parameters."""
    with open(path, "r") as f:
        s = f.read()
    return load_string(s, os.path.dirname(os.path.abspath(path)), **params)
