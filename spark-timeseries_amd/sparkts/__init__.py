"""sparkts -- MI355X-native host mirror of spark-timeseries' series-wise hot path.

Module and class names follow the reference (com.cloudera.sparkts.*):
  UnivariateTimeSeries  fillts / fill* / autocorr / lag / differencesAtLag / ar
  models                EWMAModel, ARModel, Autoregression
  TimeSeriesRDD         fill / mapSeries over a keyed panel (one shard per rank)
Every operator runs as a batched HIP kernel through libsts_hip.so (include/sts.h);
there is no CPU fallback.
"""
from . import UnivariateTimeSeries  # noqa: F401
from .errors import (DeviceError, IllegalArgumentException, MathIllegalArgumentException,  # noqa: F401
                     NullPointerException, SingularMatrixException, TooManyEvaluationsException,
                     TooManyIterationsException, UnsupportedOperationException)
from .timeseriesrdd import TimeSeriesRDD  # noqa: F401
