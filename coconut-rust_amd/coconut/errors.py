"""Error kinds — mirror reference src/errors.rs:6-24 (CoconutErrorKind) and the C ABI codes."""
import enum


class CoconutErrorKind(enum.Enum):
    UnsupportedNoOfMessages = -1   # errors.rs:8-12
    UnequalNoOfBasesExponents = -2  # errors.rs:14-18
    Threshold = -3                  # reference: assert! panic (signature.rs:449,484)
    Decode = -4
    Hip = -5
    Rccl = -6
    State = -7
    GeneralError = -100             # errors.rs:23-24


class CoconutError(Exception):
    def __init__(self, code: int, msg: str = ""):
        try:
            self.kind = CoconutErrorKind(code)
        except ValueError:
            self.kind = CoconutErrorKind.GeneralError
        self.code = code
        super().__init__(f"{self.kind.name} ({code}) {msg}".strip())
