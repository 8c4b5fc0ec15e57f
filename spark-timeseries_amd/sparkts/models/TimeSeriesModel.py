"""com.cloudera.sparkts.models.TimeSeriesModel (S/models/TimeSeriesModel.scala:23-45)."""
from __future__ import annotations


class TimeSeriesModel:
    def removeTimeDependentEffects(self, ts, dest=None):  # pragma: no cover - interface
        """Series with this model's time-dependent effects removed (returns dest)."""
        raise NotImplementedError

    def addTimeDependentEffects(self, ts, dest=None):  # pragma: no cover - interface
        """i.i.d. series with this model's time-dependent effects added (returns dest)."""
        raise NotImplementedError
