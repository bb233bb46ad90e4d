"""Read-through view of a train config with every Enum member replaced by its value string.

The reference's TrainConfig (modules/util/config/TrainConfig.py:759-995) stores enum-typed
fields as Enum members (`LossScaler.NONE`, `TimestepDistribution.UNIFORM`, `Optimizer.ADAMW`,
`ModelType.STABLE_DIFFUSION_XL_10_BASE`, `PeftType.LORA` ...), and its GenericTrainer passes that
object to every plugin call (GenericTrainer.py:688-736).  This build's own TrainConfig keeps
plain strings.  Every plugin / trainer / factory entry point wraps its `config` argument with
`plain()`, so all decisions compare strings whichever object the caller passed:

    plain(ref_cfg).loss_scaler == "NONE"          # LossScaler.NONE
    plain(ref_cfg).optimizer.optimizer == "ADAMW" # nested part configs are wrapped too

Writes go through to the wrapped object.  Build-only knobs missing from a reference config
(data-parallel bucket size / reduce dtype) read their defaults from BUILD_DEFAULTS.
"""
from __future__ import annotations

import dataclasses
from enum import Enum
from types import SimpleNamespace

BUILD_DEFAULTS = {"dp_bucket_mb": 256, "dp_reduce_fp32": False}


def _is_config(v) -> bool:
    if isinstance(v, (str, bytes, int, float, bool, list, tuple, dict)) or v is None:
        return False
    return (dataclasses.is_dataclass(v) or isinstance(v, SimpleNamespace)
            or (hasattr(v, "to_dict") and hasattr(v, "types")))


def value(v):
    """Enum member -> its value; anything else unchanged."""
    return v.value if isinstance(v, Enum) else v


class PlainConfig:
    __slots__ = ("_c",)

    def __init__(self, c):
        object.__setattr__(self, "_c", c)

    def __getattr__(self, k):
        c = object.__getattribute__(self, "_c")
        try:
            v = getattr(c, k)
        except AttributeError:
            if k in BUILD_DEFAULTS:
                return BUILD_DEFAULTS[k]
            raise
        if isinstance(v, Enum):
            return v.value
        if _is_config(v):
            return PlainConfig(v)
        return v

    def __setattr__(self, k, v):
        setattr(object.__getattribute__(self, "_c"), k, v)

    def unwrap(self):
        return object.__getattribute__(self, "_c")

    def __repr__(self):
        return f"PlainConfig({object.__getattribute__(self, '_c')!r})"


def plain(config):
    if config is None or isinstance(config, PlainConfig):
        return config
    return PlainConfig(config)
