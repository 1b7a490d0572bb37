"""ANN inverse kinematics on the GPU -- kinematics/ann.py of the reference.

ANN.predict(positions) -> float32 (n, 4) exactly as the reference's
x-scaler -> Keras Sequential -> y-scaler pipeline (ann.py:70-76), computed by
libikhip's single fused kernel (fp32 MFMA layer chain, scalers in float64).

Model files (ann.py:78-95):
  * `<name>.h5` (Keras HDF5, read by models/keras_h5.py without h5py) with the
    reference's `<name>_scaler_x.bin` / `<name>_scaler_y.bin` beside it
    (decoded by models/scaler_bin.py without unpickling);
  * save_model() writes that same layout (`<prefix>_<timestamp>.h5` through
    models/hdf5_write.py, the scalers as joblib-dumped sklearn StandardScalers)
    so the reference's load_model can open it; `<name>.npz` (weights,
    activations and scalers) is also read.
Training (ann.py:27-68) is out of scope for this engine.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from datetime import datetime
from typing import List

import numpy as np

from .. import _native
from ..models.scaler_bin import ScalerParams, load_scaler


@dataclass
class DenseModel:
    """A Keras Sequential of Dense layers: h = act(h @ W + b)."""
    weights: List[np.ndarray]
    biases: List[np.ndarray]
    activations: List[str]
    name: str = "model"
    layer_names: List[str] = field(default_factory=list)

    @property
    def dims(self):
        return [self.weights[0].shape[0]] + [w.shape[1] for w in self.weights]

    def count_params(self):
        return int(sum(w.size + b.size for w, b in zip(self.weights, self.biases)))

    def flops_per_point(self):
        return int(sum(2 * w.shape[0] * w.shape[1] for w in self.weights))


def glorot_model(dims=(3,) + (500,) * 12 + (4,), seed=0, hidden_act="tanh") -> DenseModel:
    """Random-init model of the reference architecture (ann.py:46-56: Input(3),
    12 x Dense(500, tanh), Dense(4)) with Keras' default initialisers
    (glorot_uniform kernels, zero biases)."""
    rng = np.random.default_rng(seed)
    Ws, bs, acts = [], [], []
    for i in range(len(dims) - 1):
        lim = np.sqrt(6.0 / (dims[i] + dims[i + 1]))
        Ws.append(rng.uniform(-lim, lim, (dims[i], dims[i + 1])).astype(np.float32))
        bs.append(np.zeros(dims[i + 1], np.float32))
        acts.append(hidden_act if i < len(dims) - 2 else "linear")
    return DenseModel(Ws, bs, acts, name=f"glorot_seed{seed}")


# The scalers shipped with the reference model (models/*_scaler_{x,y}.bin),
# decoded by models/scaler_bin.py; used with synthetic weights for benches.
REFERENCE_X_SCALER = ScalerParams(
    mean=np.array([2.2073088909641334, 0.19405985835497927, 1.494994275926956]),
    scale=np.array([1.7144761363570307, 2.7973201512836416, 2.140079230865925]), var=None)
REFERENCE_Y_SCALER = ScalerParams(
    mean=np.array([0.052229169532186454, 0.9236331507819656, -1.3859332319838136,
                   -0.42092474514907724]),
    scale=np.array([0.8768847052996848, 0.6520665510519178, 1.0214536342625566,
                    0.4481255851377674]), var=None)


def load_npz_model(path):
    with np.load(path, allow_pickle=False) as z:
        nl = int(z["n_layers"])
        Ws = [z[f"W{i}"].astype(np.float32) for i in range(nl)]
        bs = [z[f"b{i}"].astype(np.float32) for i in range(nl)]
        acts = [str(a) for a in z["acts"]]
        xs = ScalerParams(mean=z["x_mean"], scale=z["x_scale"], var=None)
        ys = ScalerParams(mean=z["y_mean"], scale=z["y_scale"], var=None)
    return DenseModel(Ws, bs, acts, name=os.path.basename(path)), xs, ys


def save_npz_model(path, model: DenseModel, xs: ScalerParams, ys: ScalerParams):
    arrs = {f"W{i}": w for i, w in enumerate(model.weights)}
    arrs.update({f"b{i}": b for i, b in enumerate(model.biases)})
    np.savez(path, n_layers=np.int32(len(model.weights)),
             acts=np.array(model.activations, dtype="<U16"), x_mean=xs.mean, x_scale=xs.scale,
             y_mean=ys.mean, y_scale=ys.scale, **arrs)


def as_features(position) -> np.ndarray:
    """The n x 3 float64 batch ANN.predict scales (ann.py:73): a single point
    (3,) is one row; any other width fails like the reference's StandardScaler
    (sklearn's feature-count check), never by reinterpreting the numbers."""
    pts = np.asarray(position, dtype=np.float64)
    if pts.ndim == 1 and pts.shape[0] == 3:
        pts = pts.reshape(1, 3)
    if pts.ndim == 2 and pts.shape[0] == 0:
        return np.empty((0, 3), np.float64)
    if pts.ndim != 2:
        raise ValueError(f"Expected 2D array, got {pts.ndim}D array instead")
    if pts.shape[1] != 3:
        raise ValueError(f"X has {pts.shape[1]} features, but StandardScaler is expecting 3 "
                         "features as input.")
    return np.ascontiguousarray(pts)


class ANN:
    """ANN class implementing the neural-network IK approach (ann.py:18-25)."""

    def __init__(self, effector_workspace_limits, dh_matrix):
        self.effector_workspace_limits = effector_workspace_limits
        self.dh_matrix = dh_matrix
        self.model = None
        self.x_data_skaler = None
        self.y_data_skaler = None
        self._uploaded_to = None

    def train_model(self, epochs, samples, features):
        raise NotImplementedError("ANN training (kinematics/ann.py:27-68) is not part of the "
                                  "MI355X inference engine; train with the reference and load "
                                  "the saved .h5 with load_model()")

    def set_model(self, model: DenseModel, x_scaler: ScalerParams, y_scaler: ScalerParams):
        """Install an in-memory model (e.g. glorot_model()) and its scalers."""
        self.model = model
        self.x_data_skaler = x_scaler
        self.y_data_skaler = y_scaler
        self._uploaded_to = None
        return self.model

    def _ctx(self):
        ctx = _native.context()
        if self.model is None:
            raise RuntimeError("no model loaded: call load_model() first")
        if self._uploaded_to is not ctx or getattr(ctx, "_ann_owner", None) is not self:
            xm, xs = self.x_data_skaler.effective()
            ym, ys = self.y_data_skaler.effective()
            ctx.ann_load(self.model.weights, self.model.biases, self.model.activations,
                         xm, xs, ym, ys)
            self._uploaded_to = ctx
            ctx._ann_owner = self
        return ctx

    def predict(self, position):
        """Scale input, run the network, rescale output (ann.py:70-76); no limit check."""
        pts = as_features(position)
        ang, _, _ = self._ctx().ann_solve(pts, check_limits=False)
        return ang

    def predict_checked(self, pts):
        """predict + the workspace check of AnnInverseKinematics.ikine (one launch)."""
        ang, _, st = self._ctx().ann_solve(pts, check_limits=True)
        return ang, st

    def predict_with_fk_error(self, position):
        """(angles, |FK(angles) - p|_2 per point, stats) -- the cli.py:54-61 round trip."""
        pts = as_features(position)
        ang, err, st = self._ctx().ann_solve(pts, check_limits=False, want_fk_err=True)
        return ang, err, st

    def load_model(self, model_h5):
        """Load model from file (ann.py:78-85)."""
        if model_h5.endswith(".npz"):
            model, xs, ys = load_npz_model(model_h5)
        else:
            from ..models.keras_h5 import load_keras_dense_model
            model = load_keras_dense_model(model_h5)
            modelname = model_h5[:-3]
            xs = load_scaler(f'{modelname}_scaler_x.bin')
            ys = load_scaler(f'{modelname}_scaler_y.bin')
        self.set_model(model, xs, ys)
        return self.model

    def save_model(self, prefix='model'):
        """Save model to `<prefix>_<timestamp>.h5` plus `..._scaler_x.bin` /
        `..._scaler_y.bin` (ann.py:87-95); returns the .h5 path."""
        from ..models.keras_h5 import save_keras_dense_model
        from ..models.scaler_bin import save_scaler
        timestamp_str = str(datetime.timestamp(datetime.now())).replace('.', '-')
        base = f'{prefix}_{timestamp_str}'
        save_keras_dense_model(f'{base}.h5', self.model)
        save_scaler(f'{base}_scaler_x.bin', self.x_data_skaler)
        save_scaler(f'{base}_scaler_y.bin', self.y_data_skaler)
        return f'{base}.h5'
