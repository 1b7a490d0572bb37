"""Read a Keras Sequential-of-Dense `.h5` model (the format ANN.save_model
writes, kinematics/ann.py:92, and ANN.load_model reads, ann.py:80) without
h5py or keras, using the minimal HDF5 parser in hdf5_min.py.

The architecture comes from the `model_config` JSON attribute (Sequential:
InputLayer + Dense layers with `units`, `activation`, `use_bias`), the weights
from `model_weights/<layer>/<weight_names...>` in `layer_names` order.
"""
from __future__ import annotations

import json

import numpy as np

from .hdf5_min import Hdf5Error, as_str, open_file

SUPPORTED_ACTS = {"linear", "tanh", "relu", "sigmoid", None}


def load_keras_dense_model(path: str):
    from ..kinematics.ann import DenseModel  # local import: avoid a cycle
    f = open_file(path)
    attrs = f.attrs
    cfg_raw = as_str(attrs.get("model_config"))
    if cfg_raw is None:
        raise Hdf5Error(f"{path}: no model_config attribute (weights-only file?)")
    cfg = json.loads(cfg_raw)
    layers = cfg["config"]["layers"] if isinstance(cfg["config"], dict) else cfg["config"]
    dense = []
    for L in layers:
        cn = L["class_name"]
        if cn in ("InputLayer",):
            continue
        if cn != "Dense":
            raise Hdf5Error(f"{path}: layer class {cn} is not supported (Dense only)")
        c = L["config"]
        act = c.get("activation", "linear")
        if isinstance(act, dict):  # serialized activation object
            act = act.get("config", {}).get("name") or act.get("class_name")
        if act not in SUPPORTED_ACTS:
            raise Hdf5Error(f"{path}: activation {act!r} is not supported")
        dense.append((c["name"], int(c["units"]), act or "linear", c.get("use_bias", True)))

    mw = f["model_weights"] if "model_weights" in f else f
    names = [as_str(n) for n in np.atleast_1d(mw.attrs.get("layer_names", []))]
    by_name = {}
    for ln in names:
        g = mw[ln]
        wn = [as_str(n) for n in np.atleast_1d(g.attrs.get("weight_names", []))]
        by_name[ln] = [g[w].read() for w in wn]

    Ws, bs, acts, lnames = [], [], [], []
    for name, units, act, use_bias in dense:
        if name not in by_name:
            raise Hdf5Error(f"{path}: no weights for layer {name}")
        arrs = by_name[name]
        W = np.asarray(arrs[0], np.float32)
        b = (np.asarray(arrs[1], np.float32) if use_bias and len(arrs) > 1
             else np.zeros(units, np.float32))
        if W.ndim != 2 or W.shape[1] != units or b.shape != (units,):
            raise Hdf5Error(f"{path}: layer {name} weight shapes {W.shape}/{b.shape} "
                            f"do not match units={units}")
        Ws.append(W)
        bs.append(b)
        acts.append(act)
        lnames.append(name)
    for i in range(1, len(Ws)):
        if Ws[i].shape[0] != Ws[i - 1].shape[1]:
            raise Hdf5Error(f"{path}: layer {lnames[i]} input width mismatch")
    return DenseModel(Ws, bs, acts, name=path, layer_names=lnames)


def _dense_config(name: str, units: int, act: str) -> dict:
    return {"name": name, "trainable": True, "dtype": "float32", "units": int(units),
            "activation": act, "use_bias": True,
            "kernel_initializer": {"class_name": "GlorotUniform", "config": {"seed": None}},
            "bias_initializer": {"class_name": "Zeros", "config": {}},
            "kernel_regularizer": None, "bias_regularizer": None,
            "activity_regularizer": None, "kernel_constraint": None, "bias_constraint": None}


def save_keras_dense_model(path: str, model, keras_version: str = "2.11.0"):
    """Write `model` (a DenseModel) as Keras' model.save('*.h5') lays out a
    Sequential of Dense layers (ann.py:46-56,92): root attributes backend /
    keras_version / model_config (JSON), `model_weights` with `layer_names`, one
    group per layer with `weight_names` and the float32 datasets at
    `<layer>/<layer>/kernel:0` and `bias:0`.  No h5py: models/hdf5_write.py."""
    from . import hdf5_write as W
    dims = model.dims
    names = (list(model.layer_names) if len(model.layer_names) == len(model.weights)
             and len(set(model.layer_names)) == len(model.weights)
             and all(n and "/" not in n for n in model.layer_names)
             else ["dense"] + [f"dense_{i}" for i in range(1, len(model.weights))])
    layers = [{"class_name": "InputLayer",
               "config": {"batch_input_shape": [None, int(dims[0])], "dtype": "float32",
                          "sparse": False, "ragged": False, "name": "input_1"}}]
    layers += [{"class_name": "Dense", "config": _dense_config(nm, dims[i + 1], act)}
               for i, (nm, act) in enumerate(zip(names, model.activations))]
    cfg = {"class_name": "Sequential", "config": {"name": "sequential", "layers": layers}}
    root = W.Group()
    root.attrs["backend"] = "tensorflow"
    root.attrs["keras_version"] = keras_version
    root.attrs["model_config"] = json.dumps(cfg)
    mw = root.group("model_weights")
    mw.attrs["backend"] = "tensorflow"
    mw.attrs["keras_version"] = keras_version
    mw.attrs["layer_names"] = names
    for nm, w, b in zip(names, model.weights, model.biases):
        g = mw.group(nm)
        wn = [f"{nm}/kernel:0", f"{nm}/bias:0"]
        g.attrs["weight_names"] = wn
        g.dataset(wn[0], np.asarray(w, np.float32))
        g.dataset(wn[1], np.asarray(b, np.float32).reshape(-1))
    W.write(path, root)
    return path
