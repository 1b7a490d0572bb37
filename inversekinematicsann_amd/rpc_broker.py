"""RPC front-end -- the reference's rpc_broker.py JSON contract on the GPU engine.

SURVEY 8(f) rank 4.  The reference serves `{"positions": [[x, y, z], ...]}`
requests from a RabbitMQ queue and answers `{"status": "OK", "angles": [...]}`
or `{"status": "ERROR", "reason": str(e), "correlation_id": id}`
(rpc_broker.py:70-100).  The payload logic is `IkineRequestHandler.handle`,
transport-free and testable on its own; `IkineRPCBroker` is the same consumer
(queue `ikine_queue` on host `rabbit_mq`, prefetch 1) and needs the `pika`
client, which is optional: without it the broker refuses to start, the
handler still works.  The engine is this package's `kinematics.inverse`
classes, so every request is one batched GPU solve.

    python -m inversekinematicsann_amd.rpc_broker --method fabrik
    python -m inversekinematicsann_amd.rpc_broker --method ann --model M.h5
"""
from __future__ import annotations

import argparse
import json
import os
import sys

from inversekinematicsann_amd.kinematics.inverse import (AnnInverseKinematics,
                                                         FabrikInverseKinematics)
from inversekinematicsann_amd.kinematics.point import Point
from inversekinematicsann_amd.robot.robot import OutOfRobotReachException
from inversekinematicsann_amd.robot.robot import SixDOFRobot as Robot

DEBUG_MSG = False


def debug_msg_print(msg):
    if DEBUG_MSG:
        print(msg)


def get_ikine_engine_cli(argv=None):
    """rpc_broker.py:26-54: `--method {ann,fabrik}` (+ `--model` for ann)."""
    p = argparse.ArgumentParser(prog="cli")
    p.add_argument("--method", required=True, type=str, choices=["ann", "fabrik"],
                   help="select inverse kinematics method, Neural Network or Fabrik")
    known, _ = p.parse_known_args(argv)
    if known.method == "ann":
        p.add_argument("--model", type=str, required=True,
                       help="select .h5 file with saved model, required only if ann ikine "
                            "method was choosed")
    args = p.parse_args(argv)
    if args.method == "ann":
        engine = AnnInverseKinematics(Robot.dh_matrix, Robot.links_lengths,
                                      Robot.effector_workspace_limits)
        engine.load_model(args.model)
        return engine
    return FabrikInverseKinematics(Robot.dh_matrix, Robot.links_lengths,
                                   Robot.effector_workspace_limits)


def exception_response(status, reason, corr_id):
    """rpc_broker.py:68-72."""
    return {"status": status, "reason": reason, "correlation_id": corr_id}


class IkineRequestHandler:
    """The body of the reference's callback (rpc_broker.py:74-92): request bytes
    in, response bytes out.  OutOfRobotReachException, ValueError (including a
    malformed JSON body or a point that is not 3 numbers) and TypeError become
    an ERROR response; anything else (ZeroDivisionError at (0, 0, 2), a body
    without "positions") propagates, as in the reference."""

    def __init__(self, ikine):
        self.ikine = ikine

    def handle(self, body: bytes, correlation_id=None) -> bytes:
        try:
            positions_json = json.loads(body.decode())
            positions = [Point(x) for x in positions_json["positions"]]
            angles_dict = dict()
            angles = self.ikine.ikine(positions)
        except (OutOfRobotReachException, ValueError, TypeError) as exception:
            debug_msg_print(str(exception))
            angles_dict = exception_response("ERROR", str(exception), correlation_id)
        else:
            angles_dict["status"] = "OK"
            angles_dict["angles"] = angles
        return json.dumps(angles_dict).encode()


class IkineRPCBroker:
    """rpc_broker.py:57-104 on the GPU engine (requires the pika client)."""

    def __init__(self, ikine, host_ip="rabbit_mq", queue_name="ikine_queue"):
        try:
            from pika import BasicProperties, BlockingConnection, ConnectionParameters
        except ImportError as e:  # transport is optional; the handler is not
            raise RuntimeError("IkineRPCBroker needs the 'pika' RabbitMQ client, which is not "
                               "installed; IkineRequestHandler serves the same payloads") from e
        self._props = BasicProperties
        self._handler = IkineRequestHandler(ikine)
        self._connection = BlockingConnection(ConnectionParameters(host=host_ip))
        self._channel = self._connection.channel()
        self._channel.queue_declare(queue=queue_name)
        self._channel.basic_qos(prefetch_count=1)
        self._channel.basic_consume(queue=queue_name, on_message_callback=self.callback)

    def callback(self, chan, method, props, body):
        resp = self._handler.handle(body, props.correlation_id)
        chan.basic_publish(exchange="", routing_key=props.reply_to,
                           properties=self._props(correlation_id=props.correlation_id),
                           body=resp)
        chan.basic_ack(delivery_tag=method.delivery_tag)

    def start(self):
        self._channel.start_consuming()


def main(argv=None):
    try:
        broker = IkineRPCBroker(get_ikine_engine_cli(argv))
        broker.start()
    except KeyboardInterrupt:
        print("CTRL+C interrupted")
        try:
            sys.exit(0)
        except SystemExit:
            os._exit(0)


if __name__ == "__main__":
    main()
