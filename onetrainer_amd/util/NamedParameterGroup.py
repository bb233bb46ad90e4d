"""Parameter groups (mirrors modules/util/NamedParameterGroup.py:9-68)."""
from __future__ import annotations


class NamedParameterGroup:
    def __init__(self, unique_name: str, parameters, learning_rate: float | None = None,
                 display_name: str | None = None):
        self.unique_name = unique_name
        self.display_name = display_name if display_name is not None else unique_name
        self.parameters = list(parameters)
        self.learning_rate = learning_rate


class NamedParameterGroupCollection:
    def __init__(self):
        self.groups: list[NamedParameterGroup] = []

    def add_group(self, g: NamedParameterGroup):
        self.groups.append(g)

    def parameters(self):
        return [p for g in self.groups for p in g.parameters]

    def parameters_for_optimizer(self, config):
        """per-group lr (NamedParameterGroup.py:36-60): the group's lr or the global one, times
        sqrt(batch_size * gradient_accumulation_steps) as config.learning_rate_scaler selects."""
        scaler = str(getattr(config, "learning_rate_scaler", "NONE"))
        bs = 1 if scaler in ("NONE", "GRADIENT_ACCUMULATION") else config.batch_size
        gas = 1 if scaler in ("NONE", "BATCH") else config.gradient_accumulation_steps
        out = []
        for g in self.groups:
            lr = g.learning_rate if g.learning_rate is not None else config.learning_rate
            lr = lr * ((bs * gas) ** 0.5)
            out.append({"params": g.parameters, "lr": lr, "initial_lr": lr})
        return out

    def unique_name_mapping(self):
        return [g.unique_name for g in self.groups]

    def display_name_mapping(self):
        return [g.display_name for g in self.groups]
