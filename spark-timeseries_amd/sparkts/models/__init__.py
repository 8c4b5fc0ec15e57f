"""com.cloudera.sparkts.models (hot-path subset: EWMA, Autoregression, ARIMA(p, d, 0), GARCH / ARGARCH)."""
from .Autoregression import ARModel, Autoregression  # noqa: F401
from .EWMA import EWMA, EWMAModel  # noqa: F401
from .TimeSeriesModel import TimeSeriesModel  # noqa: F401
from .ARIMA import ARIMA, ARIMAModel  # noqa: F401
from .GARCH import ARGARCH, ARGARCHModel, GARCH, GARCHModel  # noqa: F401
