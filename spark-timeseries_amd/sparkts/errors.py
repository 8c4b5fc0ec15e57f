"""JVM exception classes of the reference, raised for the C-ABI status codes.

The reference signals errors with JVM exceptions; the host
mirror raises same-named Python exceptions with the reference's messages so code
and tests written against the reference read the same.
"""
from __future__ import annotations

STS_OK = 0
STS_ERR_BAD_ARG = 1
STS_ERR_ALL_NAN = 2
STS_ERR_UNSUPPORTED_METHOD = 3
STS_ERR_HIP = 4
STS_ERR_REQUIREMENT = 5
STS_ERR_NULL_DEST = 6
STS_ERR_NOT_ENOUGH_DATA = 7
STS_ERR_SINGULAR = 8
STS_ERR_NO_DEVICE = 9
STS_ERR_TOO_MANY_EVALUATIONS = 10
STS_ERR_TOO_MANY_ITERATIONS = 11
STS_ERR_TOO_FEW_POINTS = 12


class IllegalArgumentException(ValueError):
    """java.lang.IllegalArgumentException (fillNearest all-NaN, require(...) failures)."""


class UnsupportedOperationException(NotImplementedError):
    """java.lang.UnsupportedOperationException (fillts with an unknown method, :148)."""


class NullPointerException(TypeError):
    """java.lang.NullPointerException (EWMAModel with dest = null, EWMA.scala:125-136)."""


class MathIllegalArgumentException(ValueError):
    """commons-math3 MathIllegalArgumentException (NOT_ENOUGH_DATA_FOR_NUMBER_OF_PREDICTORS)."""


class SingularMatrixException(ArithmeticError):
    """commons-math3 SingularMatrixException."""


class TooManyEvaluationsException(RuntimeError):
    """commons-math3 TooManyEvaluationsException (EWMA.fitModel: MaxEval 10000 exceeded)."""


class TooManyIterationsException(RuntimeError):
    """commons-math3 TooManyIterationsException (EWMA.fitModel: MaxIter 10000 exceeded)."""


class NumberIsTooSmallException(ValueError):
    """commons-math3 NumberIsTooSmallException (fillSpline: SplineInterpolator needs at least
    3 non-NaN values, NUMBER_OF_POINTS)."""


class DeviceError(RuntimeError):
    """HIP runtime failure or no gfx950 device (the engine has no CPU fallback)."""


def _message() -> str:
    from ._native import lib
    m = lib().sts_last_error()
    return m.decode() if m else ""


def raise_for_status(status: int, what: str = "") -> None:
    if status == STS_OK:
        return
    msg = _message() or what
    if status == STS_ERR_ALL_NAN:
        raise IllegalArgumentException("Input is all NaNs!")
    if status == STS_ERR_REQUIREMENT:
        raise IllegalArgumentException(msg)
    if status == STS_ERR_UNSUPPORTED_METHOD:
        raise UnsupportedOperationException(msg)
    if status == STS_ERR_NULL_DEST:
        raise NullPointerException(msg)
    if status == STS_ERR_NOT_ENOUGH_DATA:
        raise MathIllegalArgumentException(msg)
    if status == STS_ERR_SINGULAR:
        raise SingularMatrixException(msg)
    if status == STS_ERR_BAD_ARG:
        raise IllegalArgumentException(msg)
    if status == STS_ERR_TOO_MANY_EVALUATIONS:
        raise TooManyEvaluationsException(msg)
    if status == STS_ERR_TOO_MANY_ITERATIONS:
        raise TooManyIterationsException(msg)
    if status == STS_ERR_TOO_FEW_POINTS:
        raise NumberIsTooSmallException(msg)
    raise DeviceError("%s (status %d)" % (msg, status))
