"""Commands a UI / script sends to a running train loop (modules/util/commands/TrainCommands.py).

The train loop polls them between steps: stop (checked after every step and epoch), backup and
save (executed at the next optimizer-update boundary, GenericTrainer.py:653-668).  The sample
commands are accepted and dropped: sampling is outside this build's hot path.  `reset()` keeps a
pending stop, as the reference does.
"""
from __future__ import annotations


class TrainCommands:
    def __init__(self, on_command=None):
        self._on_command = on_command
        self._stop = False
        self.reset()

    def reset(self):
        self._flags = {"backup": False, "save": False, "sample_default": False}
        self._sample_custom: list = []

    def set_on_command(self, on_command):
        self._on_command = on_command

    def get_and_reset_on_command(self):
        cb, self._on_command = self._on_command, None
        return cb

    def _notify(self):
        if self._on_command:
            self._on_command(self)

    def _take(self, key: str) -> bool:
        v, self._flags[key] = self._flags[key], False
        return v

    def stop(self):
        self._stop = True
        self._notify()

    def get_stop_command(self) -> bool:
        return self._stop

    def backup(self):
        self._flags["backup"] = True
        self._notify()

    def get_and_reset_backup_command(self) -> bool:
        return self._take("backup")

    def save(self):
        self._flags["save"] = True
        self._notify()

    def get_and_reset_save_command(self) -> bool:
        return self._take("save")

    def sample_default(self):
        self._flags["sample_default"] = True
        self._notify()

    def get_and_reset_sample_default_command(self) -> bool:
        return self._take("sample_default")

    def sample_custom(self, sample_params):
        self._sample_custom.append(sample_params)
        self._notify()

    def get_and_reset_sample_custom_commands(self) -> list:
        out, self._sample_custom = self._sample_custom, []
        return out
