"""Serving error codes (TF-Serving / gRPC status semantics)."""
from __future__ import annotations

import enum


class Code(enum.IntEnum):
    OK = 0
    CANCELLED = 1
    UNKNOWN = 2
    INVALID_ARGUMENT = 3
    DEADLINE_EXCEEDED = 4
    NOT_FOUND = 5
    FAILED_PRECONDITION = 9
    RESOURCE_EXHAUSTED = 8
    UNIMPLEMENTED = 12
    INTERNAL = 13
    UNAVAILABLE = 14


class ServingError(Exception):
    def __init__(self, code: Code, message: str):
        super().__init__(f"{code.name}: {message}")
        self.code = code
        self.message = message

    def grpc_code(self):
        import grpc

        return getattr(grpc.StatusCode, self.code.name)
