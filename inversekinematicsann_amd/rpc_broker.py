"""RPC service: batched IK requests over a RabbitMQ request/reply queue.

The wire contract is the reference's (rpc_broker.py:57-104),
kept byte-compatible with its clients (examples/rpc_client.py):

    request  {"positions": [[x, y, z], ...]}
    reply    {"status": "OK", "angles": [[t1, t2, t3, t4], ...]}
          or {"status": "ERROR", "reason": "<exception text>", "correlation_id": <id>}

on queue "ikine_queue" of host "rabbit_mq", one unacknowledged request at a
time.  A request is one batched GPU solve through this package's
kinematics.inverse engines.  `IkineRequestHandler` is the transport-free part
(bytes in, bytes out); `IkineRPCBroker` binds it to RabbitMQ and needs the
optional `pika` client.

    python -m inversekinematicsann_amd.rpc_broker --method fabrik
    python -m inversekinematicsann_amd.rpc_broker --method ann --model M.h5
"""
from __future__ import annotations

import argparse
import json
import logging
from typing import List, Optional, Sequence

from inversekinematicsann_amd.kinematics.inverse import (AnnInverseKinematics,
                                                         FabrikInverseKinematics)
from inversekinematicsann_amd.kinematics.point import Point
from inversekinematicsann_amd.robot.robot import OutOfRobotReachException
from inversekinematicsann_amd.robot.robot import SixDOFRobot as Robot

RPC_HOST = "rabbit_mq"
RPC_QUEUE = "ikine_queue"

# What a bad request can raise and the client gets back as an ERROR reply: a
# point out of reach, a malformed body or point (json / Point), a non-list
# "positions".  Anything else (a body without "positions", ZeroDivisionError at
# the base-top joint) is a fault of the service and propagates, as it does in
# the reference.
REPLY_ERRORS = (OutOfRobotReachException, ValueError, TypeError)

log = logging.getLogger("ikhip.rpc")


def decode_request(body: bytes) -> List[Point]:
    return [Point(p) for p in json.loads(body.decode())["positions"]]


def ok_reply(angles) -> dict:
    return {"status": "OK", "angles": angles}


def error_reply(exc: BaseException, correlation_id) -> dict:
    return {"status": "ERROR", "reason": str(exc), "correlation_id": correlation_id}


class IkineRequestHandler:
    """One request body -> one reply body, through an engine with ikine()."""

    def __init__(self, ikine):
        self.ikine = ikine

    def handle(self, body: bytes, correlation_id=None) -> bytes:
        try:
            reply = ok_reply(self.ikine.ikine(decode_request(body)))
        except REPLY_ERRORS as exc:
            log.debug("request %s refused: %s", correlation_id, exc)
            reply = error_reply(exc, correlation_id)
        return json.dumps(reply).encode()


def build_engine(method: str, model: Optional[str] = None):
    """The SixDOFRobot engine of `method` (with `model` loaded for ann)."""
    if method == "ann":
        engine = AnnInverseKinematics(Robot.dh_matrix, Robot.links_lengths,
                                      Robot.effector_workspace_limits)
        engine.load_model(model)
        return engine
    return FabrikInverseKinematics(Robot.dh_matrix, Robot.links_lengths,
                                   Robot.effector_workspace_limits)


def get_ikine_engine_cli(argv: Optional[Sequence[str]] = None):
    """The engine named on the command line: --method {ann,fabrik} [--model M.h5]."""
    parser = argparse.ArgumentParser(prog="rpc_broker",
                                     description="serve IK requests from a RabbitMQ queue")
    parser.add_argument("--method", required=True, choices=["ann", "fabrik"],
                        help="IK engine behind the queue")
    parser.add_argument("--model", help="Keras .h5 model (with its _scaler_x/_y.bin files); "
                                        "needed by --method ann")
    args = parser.parse_args(argv)
    if args.method == "ann" and not args.model:
        parser.error("--method ann needs --model")
    return build_engine(args.method, args.model)


class IkineRPCBroker:
    """RabbitMQ consumer of RPC_QUEUE: each request is answered on its reply_to
    queue with the same correlation id, then acknowledged (prefetch 1)."""

    def __init__(self, ikine, host_ip: str = RPC_HOST, queue_name: str = RPC_QUEUE):
        try:
            import pika
        except ImportError as e:  # the transport is optional, the handler is not
            raise RuntimeError("IkineRPCBroker needs the 'pika' RabbitMQ client, which is not "
                               "installed; IkineRequestHandler serves the same payloads") from e
        self._pika = pika
        self.handler = IkineRequestHandler(ikine)
        self.connection = pika.BlockingConnection(pika.ConnectionParameters(host=host_ip))
        self.channel = self.connection.channel()
        self.channel.queue_declare(queue=queue_name)
        self.channel.basic_qos(prefetch_count=1)
        self.channel.basic_consume(queue=queue_name, on_message_callback=self._on_request)

    def _on_request(self, channel, delivery, props, body):
        reply = self.handler.handle(body, props.correlation_id)
        channel.basic_publish(exchange="", routing_key=props.reply_to, body=reply,
                              properties=self._pika.BasicProperties(
                                  correlation_id=props.correlation_id))
        channel.basic_ack(delivery_tag=delivery.delivery_tag)

    def serve(self):
        self.channel.start_consuming()

    start = serve

    def close(self):
        """Stop consuming and close; quiet when pika already closed the
        connection (an interrupt can land in its I/O loop)."""
        for step in (self.channel.stop_consuming, self.connection.close):
            try:
                step()
            except Exception as e:  # noqa: BLE001 -- closing is best effort
                log.debug("close: %s: %s", step.__name__, e)


def main(argv: Optional[Sequence[str]] = None) -> int:
    """Start the broker; Ctrl+C at any point (model load, connect, serving) exits
    cleanly with status 0, as the reference's main does (rpc_broker.py:107-119)."""
    broker = None
    try:
        broker = IkineRPCBroker(get_ikine_engine_cli(argv))
        broker.serve()
    except KeyboardInterrupt:
        log.info("interrupted; closing the connection")
        print("CTRL+C interrupted")
        if broker is not None:
            broker.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
