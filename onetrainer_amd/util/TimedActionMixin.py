"""Step / epoch / wall-clock action timers of the train loop.

Restates modules/util/TimedActionMixin.py:13-103 (repeating_action_needed, single_action_elapsed),
which GenericTrainer uses for backup_after / save_every / save_skip_first / the 5-minute gc
(modules/trainer/GenericTrainer.py:506-523).  Units are the TimeUnit values as strings (the
reference's enum goes through util/config/plain.py).
"""
from __future__ import annotations

import time

_SECONDS = {"SECOND": 1.0, "MINUTE": 60.0, "HOUR": 3600.0}


class TimedActionMixin:
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._last_action: dict[str, float] = {}
        self._start_time = time.time()

    @staticmethod
    def _unit(unit) -> str:
        return str(getattr(unit, "value", unit))

    def repeating_action_needed(self, name: str, interval: float, unit, train_progress,
                                start_at_zero: bool = True) -> bool:
        """TimedActionMixin.py:13-72.  STEP / EPOCH count on the train progress (with start_at_zero
        False the action fires at the END of each interval: global_step + 1, and epochs only after
        the first); SECOND / MINUTE / HOUR are wall-clock intervals since the previous firing (with
        start_at_zero False the clock starts at the first query instead of firing at once)."""
        unit = self._unit(unit)
        last = self._last_action.setdefault(name, -1.0)
        if unit == "EPOCH":
            hit = train_progress.epoch % int(interval) == 0 and train_progress.epoch_step == 0
            return hit and (start_at_zero or train_progress.epoch > 0)
        if unit == "STEP":
            step = train_progress.global_step if start_at_zero else train_progress.global_step + 1
            return step % int(interval) == 0
        if unit in _SECONDS:
            now = time.time()
            if not start_at_zero and last < 0:
                self._last_action[name] = last = now
            if now - last > interval * _SECONDS[unit]:
                self._last_action[name] = now
                return True
            return False
        return unit == "ALWAYS"   # NEVER (and anything unknown) never fires

    def single_action_elapsed(self, name: str, delay: float, unit, train_progress) -> bool:
        """TimedActionMixin.py:74-103: has `delay` elapsed since the start (epochs / steps counted
        one-based, wall clock since the trainer was built)?"""
        unit = self._unit(unit)
        self._last_action.setdefault(name, time.time())
        if unit == "EPOCH":
            return train_progress.epoch + 1 > int(delay)
        if unit == "STEP":
            return train_progress.global_step + 1 > int(delay)
        if unit in _SECONDS:
            return time.time() - self._start_time > delay * _SECONDS[unit]
        return unit == "ALWAYS"
