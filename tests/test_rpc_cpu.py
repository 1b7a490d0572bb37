"""RPC payload contract (reference rpc_broker.py:57-104) with a stand-in engine:
the response bytes, which exceptions become ERROR responses and which
propagate.  The GPU engine behind the same handler: tests/test_gpu_cli.py."""
import json

import pytest

from inversekinematicsann_amd.robot.robot import OutOfRobotReachException


class _Engine:
    def __init__(self, result=None, exc=None):
        self.result, self.exc, self.seen = result, exc, None

    def ikine(self, positions):
        self.seen = positions
        if self.exc is not None:
            raise self.exc
        return self.result


def _handler(engine):
    from inversekinematicsann_amd.rpc_broker import IkineRequestHandler
    return IkineRequestHandler(engine)


def test_ok_response_bytes_and_points():
    from inversekinematicsann_amd.kinematics.point import Point
    eng = _Engine(result=[[0.5, 1.0, -1.25, 2.0], [0.0, 0.1, 0.2, 0.3]])
    body = json.dumps({"positions": [[1.0, 2.1, 3.0], [1.5, 2.2, -2.1]]}).encode()
    out = _handler(eng).handle(body, "c-1")
    # rpc_broker.py:86-91: status first, then angles; json.dumps default separators
    assert out == json.dumps({"status": "OK", "angles": eng.result}).encode()
    assert all(isinstance(p, Point) for p in eng.seen) and eng.seen[1].z == -2.1


def test_out_of_reach_is_an_error_response():
    msg = "Inverse Kinematics exception, point Point(1.0, 2.0, -4.0) is out of manipulator " \
          "reach area! Limits: {'x': [0, 6], 'y': [-6, 6], 'z': [-3, 6]}"
    eng = _Engine(exc=OutOfRobotReachException(msg))
    out = json.loads(_handler(eng).handle(b'{"positions": [[1.0, 2.0, -4.0]]}', "abc"))
    assert out == {"status": "ERROR", "reason": msg, "correlation_id": "abc"}
    assert list(out) == ["status", "reason", "correlation_id"]  # rpc_broker.py:68-72 order


@pytest.mark.parametrize("body,reason_start", [
    (b'{"positions": [[1.0, 2.0]]}', "3D Point input shape should be (3,) not (2,)"),
    (b'not json', "Expecting value"),
    (b'{"positions": 5}', "'int' object is not iterable"),
])
def test_value_and_type_errors_are_error_responses(body, reason_start):
    out = json.loads(_handler(_Engine(result=[])).handle(body, None))
    assert out["status"] == "ERROR" and out["reason"].startswith(reason_start)
    assert out["correlation_id"] is None


@pytest.mark.parametrize("exc_body", [
    (ZeroDivisionError("float division by zero"), b'{"positions": [[0, 0, 2]]}'),
    (None, b'{"points": []}'),  # KeyError: the reference does not catch it
])
def test_other_exceptions_propagate(exc_body):
    exc, body = exc_body
    with pytest.raises((ZeroDivisionError, KeyError)):
        _handler(_Engine(result=[], exc=exc)).handle(body, "x")


def test_engine_cli_and_broker_without_pika():
    from inversekinematicsann_amd import rpc_broker
    eng = rpc_broker.get_ikine_engine_cli(["--method", "fabrik"])
    assert type(eng).__name__ == "FabrikInverseKinematics"
    with pytest.raises(SystemExit):  # --model is required for ann (rpc_broker.py:34-36)
        rpc_broker.get_ikine_engine_cli(["--method", "ann"])
    try:
        import pika  # noqa: F401
    except ImportError:
        with pytest.raises(RuntimeError, match="pika"):
            rpc_broker.IkineRPCBroker(eng)


def test_ctrl_c_during_setup_and_close_errors(monkeypatch, capsys):
    """Ctrl+C while the engine loads or the broker connects exits 0 (the
    reference's main catches it around both, rpc_broker.py:107-119), and close()
    survives a connection pika already closed."""
    from inversekinematicsann_amd import rpc_broker as R

    def interrupted(argv=None):
        raise KeyboardInterrupt
    monkeypatch.setattr(R, "get_ikine_engine_cli", interrupted)
    assert R.main(["--method", "fabrik"]) == 0
    assert "CTRL+C interrupted" in capsys.readouterr().out

    class Dead:
        def stop_consuming(self):
            raise RuntimeError("connection already closed")

        def close(self):
            raise RuntimeError("connection already closed")
    b = R.IkineRPCBroker.__new__(R.IkineRPCBroker)
    b.channel = b.connection = Dead()
    b.close()
