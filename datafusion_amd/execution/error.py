"""ExecutionError (src/execution/error.rs:27-35) as a Python exception.

``kind`` names the Rust variant the reference would return (ExecutionError,
General, NotImplemented, ArrowError(DivideByZero), ...), ``message`` its text.
``kind == "panic"`` marks paths where the reference panics instead.
"""
from .._abi import STATUS_NAMES


class ExecutionError(Exception):
    def __init__(self, kind: str, message: str, code: int = 0):
        super().__init__("%s(%r)" % (kind, message))
        self.kind = kind
        self.message = message
        self.code = code

    @staticmethod
    def from_status(code: int, message: str) -> "ExecutionError":
        return ExecutionError(STATUS_NAMES.get(code, "Unknown(%d)" % code), message, code)
