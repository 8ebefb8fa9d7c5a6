"""Minimal mmengine-style registries used when mmengine / mmdet3d are absent.

`MODELS` builds the detector stack from the reference's config dicts (`type=` strings with
kwargs, configs/adversarial/*.py); `ADVERSARIES` mirrors models/builder.py:6-11. When
mmengine and mmdet3d ARE importable, the plugin modules register into their registries
instead (robustpointclouds_amd/plugin/models/...), so the reference's configs and
train_*.py runners resolve the same type names.
"""
from __future__ import annotations

import copy


class Registry:
    def __init__(self, name, parent=None, scope=None):
        self.name = name
        self._m = {}

    def register_module(self, name=None, force=False, module=None):
        def deco(cls):
            # re-registration (the plugin package imported both as `models` and as
            # `robustpointclouds_amd.plugin.models`) replaces the entry, like force=True
            self._m[name or cls.__name__] = cls
            return cls
        if module is not None:
            return deco(module)
        return deco

    def get(self, key):
        key = key.split(".")[-1]          # 'mmdet.FocalLoss' -> 'FocalLoss'
        return self._m.get(key)

    def __contains__(self, key):
        return self.get(key) is not None

    def build(self, cfg, **default_args):
        if cfg is None:
            return None
        cfg = copy.deepcopy(dict(cfg))
        cfg.pop("_delete_", None)
        t = cfg.pop("type")
        cls = self.get(t) if isinstance(t, str) else t
        if cls is None:
            raise KeyError(f"{t} is not registered in {self.name}")
        for k, v in default_args.items():
            cfg.setdefault(k, v)
        if self.name == "hooks":
            cfg.pop("priority", None)   # consumed by mmengine's Runner.register_hook, not the hook
        return cls(**cfg)


MODELS = Registry("models")
ADVERSARIES = Registry("adversaries")
HOOKS = Registry("hooks")
