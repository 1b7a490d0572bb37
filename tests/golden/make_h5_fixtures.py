"""Write small Keras-layout .h5 model files with h5py, for the h5py-free reader
(inversekinematicsann_amd/models/keras_h5.py).

Run with the interpreter that has h5py (build container only):

    /opt/conda/bin/python3.9 tests/golden/make_h5_fixtures.py

The layout follows what Keras' `model.save('m.h5')` writes for a Sequential of
Dense layers (kinematics/ann.py:46-56,92): root attributes backend /
keras_version / model_config (JSON) / training_config, a `model_weights` group
with a `layer_names` attribute, one group per layer with a `weight_names`
attribute and the datasets at `<layer>/<layer>/kernel:0` and `bias:0`, plus an
`optimizer_weights` group.  Keras stores those string attributes as bytes
(fixed-length HDF5 strings); one file uses Python str (variable-length
strings, global heap) and one uses libver='latest' (superblock v2+, v2 object
headers, link messages) to exercise the other encodings.  The weights are
also saved to an .npz for comparison.
"""
import json
import os

import h5py
import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))


def make_model(dims, seed):
    rng = np.random.default_rng(seed)
    Ws, bs = [], []
    for i in range(len(dims) - 1):
        lim = np.sqrt(6.0 / (dims[i] + dims[i + 1]))
        Ws.append(rng.uniform(-lim, lim, (dims[i], dims[i + 1])).astype(np.float32))
        bs.append(rng.normal(0, 0.05, dims[i + 1]).astype(np.float32))
    return Ws, bs


def model_config(dims, acts, names):
    layers = [{"class_name": "InputLayer",
               "config": {"batch_input_shape": [None, dims[0]], "dtype": "float32",
                          "sparse": False, "ragged": False, "name": "input_1"}}]
    for i, (a, nm) in enumerate(zip(acts, names)):
        layers.append({"class_name": "Dense", "config": {
            "name": nm, "trainable": True, "dtype": "float32", "units": dims[i + 1],
            "activation": a, "use_bias": True,
            "kernel_initializer": {"class_name": "GlorotUniform", "config": {"seed": None}},
            "bias_initializer": {"class_name": "Zeros", "config": {}},
            "kernel_regularizer": None, "bias_regularizer": None,
            "activity_regularizer": None, "kernel_constraint": None, "bias_constraint": None}})
    return {"class_name": "Sequential", "config": {"name": "sequential", "layers": layers}}


def write(path, dims, acts, seed, as_str=False, libver="earliest"):
    Ws, bs = make_model(dims, seed)
    names = ["dense"] + [f"dense_{i}" for i in range(1, len(Ws))]
    enc = (lambda s: s) if as_str else (lambda s: s.encode("utf8"))
    with h5py.File(path, "w", libver=libver) as f:
        f.attrs["backend"] = enc("tensorflow")
        f.attrs["keras_version"] = enc("2.11.0")
        f.attrs["model_config"] = enc(json.dumps(model_config(dims, acts, names)))
        f.attrs["training_config"] = enc(json.dumps({"loss": "mse", "optimizer_config": {
            "class_name": "Adam", "config": {"learning_rate": 1e-5}}}))
        mw = f.create_group("model_weights")
        mw.attrs["backend"] = enc("tensorflow")
        mw.attrs["keras_version"] = enc("2.11.0")
        mw.attrs["layer_names"] = (np.array(names, dtype=object) if as_str
                                   else np.array([n.encode() for n in names]))
        for nm, W, b in zip(names, Ws, bs):
            g = mw.create_group(nm)
            wn = [f"{nm}/kernel:0", f"{nm}/bias:0"]
            g.attrs["weight_names"] = (np.array(wn, dtype=object) if as_str
                                       else np.array([w.encode() for w in wn]))
            g.create_dataset(wn[0], data=W)
            g.create_dataset(wn[1], data=b)
        ow = f.create_group("optimizer_weights")
        ow.create_dataset("Adam/iter:0", data=np.int64(1234))
    np.savez(path[:-3] + "_weights.npz", dims=np.array(dims), acts=np.array(acts),
             **{f"W{i}": w for i, w in enumerate(Ws)}, **{f"b{i}": b for i, b in enumerate(bs)})
    print(path)


if __name__ == "__main__":
    write(os.path.join(OUT, "keras_dense_small.h5"), (3, 16, 16, 4),
          ["tanh", "tanh", "linear"], seed=1)
    write(os.path.join(OUT, "keras_dense_vlenstr.h5"), (3, 24, 4), ["relu", "linear"], seed=2,
          as_str=True)
    write(os.path.join(OUT, "keras_dense_latest.h5"), (3, 40, 33, 4),
          ["sigmoid", "tanh", "linear"], seed=3, libver="latest")
    # the reference's depth (ann.py:46-56: 12 hidden + output) at a small width:
    # 13 layer groups -> several symbol-table nodes under one B-tree
    write(os.path.join(OUT, "keras_dense_deep.h5"), (3,) + (12,) * 12 + (4,),
          ["tanh"] * 12 + ["linear"], seed=4)
