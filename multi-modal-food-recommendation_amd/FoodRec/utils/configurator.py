"""Config cascade — same semantics as the reference's utils/configurator.py:

* files merged in order overall.yaml -> dataset/<dataset>.yaml -> model/<model>.yaml
  (-> mg.yaml when mg=True), each file's ``hyper_parameters`` lists concatenated (:64-86);
* the caller's ``config_dict`` overrides the files (:58-60);
* YAML floats written like ``1e-04`` parse as floats (custom implicit resolver, :88-100);
* ``valid_metric_bigger`` derived from valid_metric; ``seed`` appended to hyper_parameters (:102-108);
* a missing key reads as ``None`` (:121-125), which many feature flags rely on;
* device = cuda when available and use_gpu (:110-114).

Config files are searched in this package's ``configs/`` directory, then in ``./configs`` of the
current working directory (the reference's location), later files overriding earlier ones.
"""
from __future__ import annotations

import os
import re

import torch
import yaml

_PKG_CONFIGS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs")

_FLOAT_RE = re.compile(r"""^(?:
     [-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
    |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
    |\.[0-9_]+(?:[eE][-+][0-9]+)?
    |[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+\.[0-9_]*
    |[-+]?\.(?:inf|Inf|INF)
    |\.(?:nan|NaN|NAN))$""", re.X)


class _Loader(yaml.SafeLoader):
    """SafeLoader plus the reference's float resolver (no arbitrary object construction)."""


_Loader.add_implicit_resolver("tag:yaml.org,2002:float", _FLOAT_RE, list("-+0123456789."))


def load_yaml(path: str) -> dict:
    with open(path, "r", encoding="utf-8") as f:
        return yaml.load(f.read(), Loader=_Loader) or {}


class Config:
    def __init__(self, model=None, dataset=None, config_dict=None, mg=False, config_dirs=None):
        config_dict = dict(config_dict or {})
        config_dict["model"] = model
        config_dict["dataset"] = dataset
        self.config_dirs = list(config_dirs) if config_dirs is not None else \
            [_PKG_CONFIGS, os.path.join(os.getcwd(), "configs")]
        self.final_config_dict = self._load_files(config_dict, mg)
        self.final_config_dict.update(config_dict)
        self._set_default_parameters()
        self._init_device()

    def _files(self, model, dataset, mg):
        names = ["overall.yaml", os.path.join("dataset", f"{dataset}.yaml"),
                 os.path.join("model", f"{model}.yaml")]
        if mg:
            names.append("mg.yaml")
        out = []
        for name in names:
            for d in self.config_dirs:
                p = os.path.join(d, name)
                if os.path.isfile(p) and os.path.abspath(p) not in {os.path.abspath(x) for x in out}:
                    out.append(p)
        return out

    def _load_files(self, config_dict, mg):
        merged, hyper = {}, []
        for path in self._files(config_dict["model"], config_dict["dataset"], mg):
            data = load_yaml(path)
            if data.get("hyper_parameters"):
                hyper.extend(data["hyper_parameters"])
            merged.update(data)
        merged["hyper_parameters"] = hyper
        return merged

    def _set_default_parameters(self):
        d = self.final_config_dict
        vm = (d.get("valid_metric") or "NDCG@20").split("@")[0]
        d["valid_metric_bigger"] = vm.lower() not in ("rmse", "mae", "logloss")
        if "seed" not in d["hyper_parameters"]:
            d["hyper_parameters"] = d["hyper_parameters"] + ["seed"]

    def _init_device(self):
        use_gpu = self.final_config_dict.get("use_gpu")
        if use_gpu and self.final_config_dict.get("gpu_id") is not None \
                and "CUDA_VISIBLE_DEVICES" not in os.environ and "HIP_VISIBLE_DEVICES" not in os.environ:
            os.environ["CUDA_VISIBLE_DEVICES"] = str(self.final_config_dict["gpu_id"])
        self.final_config_dict["device"] = torch.device(
            "cuda" if (use_gpu and torch.cuda.is_available()) else "cpu")

    def __setitem__(self, key, value):
        if not isinstance(key, str):
            raise TypeError("index must be a str.")
        self.final_config_dict[key] = value

    def __getitem__(self, item):
        return self.final_config_dict.get(item)

    def __contains__(self, key):
        if not isinstance(key, str):
            raise TypeError("index must be a str.")
        return key in self.final_config_dict

    def get(self, key, default=None):
        v = self.final_config_dict.get(key)
        return default if v is None else v

    def __str__(self):
        return "\n" + "\n".join(f"{k}={v}" for k, v in self.final_config_dict.items()) + "\n\n"

    __repr__ = __str__
