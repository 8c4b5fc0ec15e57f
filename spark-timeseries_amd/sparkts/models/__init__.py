"""com.cloudera.sparkts.models (hot-path subset: EWMA, Autoregression)."""
from .Autoregression import ARModel, Autoregression  # noqa: F401
from .EWMA import EWMA, EWMAModel  # noqa: F401
from .TimeSeriesModel import TimeSeriesModel  # noqa: F401
