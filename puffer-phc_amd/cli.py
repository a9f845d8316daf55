"""Dotted-flag CLI over nested dataclasses (the reference parses AppConfig with tyro,
scripts/train.py:435; tyro is not available offline).  Flags follow tyro's spelling:
`--env.num-envs 4096`, `--train.batch-size 131072`, `--mode train`, `--env.use-amp-obs`
(booleans also accept `--env.use-amp-obs False` / `--env.no-use-amp-obs`)."""

import argparse
import dataclasses
import enum
import typing


def _walk(cls_or_obj, prefix=""):
    for f in dataclasses.fields(cls_or_obj):
        if not f.init:
            continue
        t = f.type
        val = getattr(cls_or_obj, f.name) if not isinstance(cls_or_obj, type) else None
        if dataclasses.is_dataclass(val):
            yield from _walk(val, prefix + f.name + ".")
        else:
            yield prefix + f.name, t, val


def _bool(s):
    if isinstance(s, bool):
        return s
    return str(s).lower() in ("1", "true", "yes", "on")


def _converter(t, default):
    origin = typing.get_origin(t)
    args = typing.get_args(t)
    if t is bool or isinstance(default, bool):
        return _bool
    if isinstance(default, enum.Enum):
        et = type(default)
        return lambda s: et[s] if s in et.__members__ else et(int(s))
    if origin is typing.Union and type(None) in args:
        inner = [a for a in args if a is not type(None)][0]
        base = _converter(inner, None)
        return lambda s: None if str(s).lower() == "none" else base(s)
    if origin is tuple or isinstance(default, tuple):
        return lambda s: tuple(int(x) for x in str(s).replace("(", "").replace(")", "").split(",") if x.strip())
    if t is int or isinstance(default, int):
        return int
    if t is float or isinstance(default, float):
        return float
    return str


def parse(cfg, argv=None):
    """Parse argv into the (already default-constructed) dataclass instance `cfg` in place."""
    ap = argparse.ArgumentParser()
    entries = list(_walk(cfg))
    for name, t, default in entries:
        flag = "--" + name.replace("_", "-")
        conv = _converter(t, default)
        if conv is _bool:
            ap.add_argument(flag, nargs="?", const=True, default=None, type=_bool, dest=name)
            parts = name.split(".")
            neg = "--" + ".".join(parts[:-1] + ["no-" + parts[-1]]).replace("_", "-")
            ap.add_argument(neg, action="store_false", dest=name)
        else:
            ap.add_argument(flag, default=None, type=conv, dest=name)
    ns = ap.parse_args(argv)
    for name, _, _ in entries:
        v = getattr(ns, name)
        if v is None:
            continue
        obj = cfg
        parts = name.split(".")
        for p in parts[:-1]:
            obj = getattr(obj, p)
        setattr(obj, parts[-1], v)
    return cfg
