"""Checkpoint format for hierarchical states.

The reference pickles the whole tree (``src/evox/core/state.py:228-234``).  Pickle
executes code on load, so evoxmi writes a single **safetensors** file instead:

* every tensor leaf is a safetensors entry keyed by a running index (``t0``, ``t1``, ...;
  version 1 keyed by the tree path, which let a dict key containing ``.`` or ``/``
  collide with another leaf); the manifest keeps the tree path of each tensor;
* the tree itself — node ids, field names, child names, Python scalars and
  dataclass type names — is a JSON manifest stored in the safetensors metadata
  under ``evoxmi_manifest`` with a ``format``/``version`` tag.

Loading never runs code from the file: dataclass node types are looked up in the
registry populated by :func:`evoxmi.core.module.dataclass` (only classes the
program itself defined can be rebuilt).  ``map_location`` places tensors.
"""
from __future__ import annotations

import dataclasses
import json
from typing import Any, Dict

import torch

FORMAT = "evoxmi-state"
VERSION = 2

_DATACLASS_REGISTRY: Dict[str, type] = {}


def register_dataclass(cls):
    _DATACLASS_REGISTRY[f"{cls.__module__}.{cls.__qualname__}"] = cls
    return cls


def _encode_value(v: Any, path: str, tensors: dict):
    from .state import State

    if isinstance(v, State):
        return {"t": "state", "node": _encode_node(v, path, tensors)}
    if isinstance(v, torch.Tensor):
        key = f"t{len(tensors)}"
        assert key not in tensors
        tensors[key] = v.detach().to("cpu").contiguous().clone()
        return {"t": "tensor", "key": key, "path": path}
    if v is None:
        return {"t": "none"}
    if isinstance(v, bool):
        return {"t": "bool", "v": v}
    if isinstance(v, int):
        return {"t": "int", "v": v}
    if isinstance(v, float):
        return {"t": "float", "v": repr(v)}
    if isinstance(v, str):
        return {"t": "str", "v": v}
    if isinstance(v, (list, tuple)):
        return {
            "t": "tuple" if isinstance(v, tuple) else "list",
            "items": [_encode_value(x, f"{path}.{i}", tensors) for i, x in enumerate(v)],
        }
    if isinstance(v, dict):
        for k in v:
            if not isinstance(k, (str, int, float, bool)):
                raise TypeError(f"cannot checkpoint dict key of type {type(k)} at {path}")
        if len({str(k) for k in v}) != len(v):
            raise ValueError(f"dict keys at {path} collide once stringified: {list(v)}")
        return {
            "t": "dict",
            "items": {str(k): _encode_value(x, f"{path}.{k}", tensors) for k, x in v.items()},
            # JSON object keys are strings: record the original key types to restore them
            "ktypes": {str(k): type(k).__name__ for k in v},
        }
    if dataclasses.is_dataclass(v):
        name = f"{type(v).__module__}.{type(v).__qualname__}"
        return {
            "t": "dataclass",
            "cls": name,
            "items": {f.name: _encode_value(getattr(v, f.name), f"{path}.{f.name}", tensors) for f in dataclasses.fields(v)},
        }
    raise TypeError(f"cannot checkpoint leaf of type {type(v)} at {path}")


def _decode_value(d: dict, tensors: dict, device):
    t = d["t"]
    if t == "state":
        return _decode_node(d["node"], tensors, device)
    if t == "tensor":
        x = tensors[d["key"]]
        return x.to(device) if device is not None else x
    if t == "none":
        return None
    if t in ("bool", "int", "str"):
        return d["v"]
    if t == "float":
        return float(d["v"])
    if t in ("tuple", "list"):
        items = [_decode_value(x, tensors, device) for x in d["items"]]
        return tuple(items) if t == "tuple" else items
    if t == "dict":
        conv = {"int": int, "float": float, "bool": lambda s: s == "True", "str": str}
        kt = d.get("ktypes", {})
        return {conv[kt.get(k, "str")](k): _decode_value(x, tensors, device) for k, x in d["items"].items()}
    if t == "dataclass":
        cls = _DATACLASS_REGISTRY.get(d["cls"])
        if cls is None:
            raise TypeError(f"dataclass {d['cls']} is not registered in this program")
        fields = {k: _decode_value(x, tensors, device) for k, x in d["items"].items()}
        obj = object.__new__(cls)
        for k, v in fields.items():
            object.__setattr__(obj, k, v)
        return obj
    raise ValueError(f"unknown manifest entry {t}")


def _encode_node(state, path: str, tensors: dict):
    from .state import State

    assert isinstance(state, State)
    sd = state._state_dict
    if dataclasses.is_dataclass(sd):
        fields = {f.name: getattr(sd, f.name) for f in dataclasses.fields(sd)}
        kind, cls = "dataclass", f"{type(sd).__module__}.{type(sd).__qualname__}"
    else:
        fields, kind, cls = sd, "dict", None
    prefix = f"{path}/" if path else ""
    return {
        "state_id": state._state_id,
        "kind": kind,
        "cls": cls,
        "fields": {k: _encode_value(v, f"{prefix}{k}", tensors) for k, v in fields.items()},
        "children": {k: _encode_node(c, f"{prefix}{k}", tensors) for k, c in state._child_states.items()},
    }


def _decode_node(node: dict, tensors: dict, device):
    from .state import State

    fields = {k: _decode_value(v, tensors, device) for k, v in node["fields"].items()}
    if node["kind"] == "dataclass":
        cls = _DATACLASS_REGISTRY.get(node["cls"])
        if cls is None:
            raise TypeError(f"dataclass {node['cls']} is not registered in this program")
        obj = object.__new__(cls)
        for k, v in fields.items():
            object.__setattr__(obj, k, v)
        sd = obj
    else:
        sd = fields
    children = {k: _decode_node(c, tensors, device) for k, c in node["children"].items()}
    st = State()._set_state_dict_mut(sd)._set_state_id_mut(node["state_id"])
    return st._set_child_states_mut(children) if children else st


def save_state(state, path: str) -> None:
    from safetensors.torch import save_file

    tensors: dict = {}
    tree = _encode_node(state, "", tensors)
    manifest = {"format": FORMAT, "version": VERSION, "tree": tree}
    save_file(tensors, path, metadata={"evoxmi_manifest": json.dumps(manifest)})


def load_state(path: str, map_location=None):
    from safetensors import safe_open

    tensors = {}
    with safe_open(path, framework="pt", device="cpu") as f:
        meta = f.metadata() or {}
        for k in f.keys():
            tensors[k] = f.get_tensor(k)
    if "evoxmi_manifest" not in meta:
        raise ValueError(f"{path} is not an evoxmi state checkpoint")
    manifest = json.loads(meta["evoxmi_manifest"])
    if manifest.get("format") != FORMAT or manifest.get("version", 0) > VERSION:
        raise ValueError(f"unsupported checkpoint format {manifest.get('format')} v{manifest.get('version')}")
    return _decode_node(manifest["tree"], tensors, map_location)
