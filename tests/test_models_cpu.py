"""Model-file readers (CPU): Keras .h5 without h5py, joblib scaler .bin
without unpickling, and the .npz round trip of ANN.save_model/load_model."""
import os
import shutil

import numpy as np
import pytest

from tests.conftest import GOLDEN

H5 = ["small", "vlenstr", "latest", "deep"]


@pytest.mark.parametrize("name", H5)
def test_keras_h5_reader_matches_h5py_written_weights(name):
    from inversekinematicsann_amd.models.keras_h5 import load_keras_dense_model
    m = load_keras_dense_model(os.path.join(GOLDEN, f"keras_dense_{name}.h5"))
    z = np.load(os.path.join(GOLDEN, f"keras_dense_{name}_weights.npz"), allow_pickle=False)
    assert m.dims == [int(d) for d in z["dims"]]
    assert m.activations == [str(a) for a in z["acts"]]
    for i in range(len(m.weights)):
        assert m.weights[i].dtype == np.float32
        assert np.array_equal(m.weights[i], z[f"W{i}"])
        assert np.array_equal(m.biases[i], z[f"b{i}"])


def test_hdf5_rejects_non_hdf5(tmp_path):
    from inversekinematicsann_amd.models.hdf5_min import Hdf5Error, open_file
    p = tmp_path / "x.h5"
    p.write_bytes(b"not an hdf5 file" * 10)
    with pytest.raises(Hdf5Error):
        open_file(str(p))


def test_ann_load_model_h5_with_reference_scalers(tmp_path):
    """ANN.load_model(<name>.h5) picks up <name>_scaler_{x,y}.bin (ann.py:81-84)."""
    from inversekinematicsann_amd.kinematics.ann import ANN
    from inversekinematicsann_amd.robot.robot import SixDOFRobot as R
    base = tmp_path / "roboarm_model"
    shutil.copy(os.path.join(GOLDEN, "keras_dense_deep.h5"), str(base) + ".h5")
    for s in "xy":
        shutil.copy(os.path.join(GOLDEN, f"roboarm_model_1674153800-982793_scaler_{s}.bin"),
                    f"{base}_scaler_{s}.bin")
    ann = ANN(R.effector_workspace_limits, R.dh_matrix)
    model = ann.load_model(str(base) + ".h5")
    assert model.dims == [3] + [12] * 12 + [4]
    assert ann.x_data_skaler.mean[0] == 2.2073088909641334
    assert ann.y_data_skaler.scale[3] == 0.4481255851377674


def test_npz_save_load_roundtrip(tmp_path):
    from inversekinematicsann_amd.kinematics.ann import (ANN, REFERENCE_X_SCALER,
                                                         REFERENCE_Y_SCALER, glorot_model)
    from inversekinematicsann_amd.robot.robot import SixDOFRobot as R
    ann = ANN(R.effector_workspace_limits, R.dh_matrix)
    ann.set_model(glorot_model((3, 7, 4), seed=3), REFERENCE_X_SCALER, REFERENCE_Y_SCALER)
    path = ann.save_model(str(tmp_path / "saved_model"))
    ann2 = ANN(R.effector_workspace_limits, R.dh_matrix)
    ann2.load_model(path)
    for a, b in zip(ann.model.weights, ann2.model.weights):
        assert np.array_equal(a, b)
    assert ann2.model.activations == ["tanh", "linear"]
    assert np.array_equal(ann2.y_data_skaler.mean, REFERENCE_Y_SCALER.mean)


def test_train_model_is_out_of_scope():
    from inversekinematicsann_amd.kinematics.ann import ANN
    with pytest.raises(NotImplementedError):
        ANN({}, []).train_model(1, [], [])
