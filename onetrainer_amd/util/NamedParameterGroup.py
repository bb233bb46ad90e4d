"""Parameter groups (mirrors modules/util/NamedParameterGroup.py:36-61)."""
from __future__ import annotations


class NamedParameterGroup:
    def __init__(self, unique_name: str, parameters, learning_rate: float | None = None):
        self.unique_name = unique_name
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
        return [{"params": g.parameters, "lr": g.learning_rate if g.learning_rate is not None else config.learning_rate,
                 "initial_lr": g.learning_rate if g.learning_rate is not None else config.learning_rate}
                for g in self.groups]

    def unique_name_mapping(self):
        return [g.unique_name for g in self.groups]
