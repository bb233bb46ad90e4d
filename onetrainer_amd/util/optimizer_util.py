"""Restoring training state after setup_model built the optimizer (the tail of
modules/util/optimizer_util.py:50-65 init_model_parameters -> create.create_optimizer, whose state
remap is create.py:1040-1086).

With a saved `param_group_mapping` each new parameter group is matched to the saved group of the
same unique name (and the same optimizer): its per-parameter state is renumbered into the new
order and the saved group's hyper-parameters are kept except `lr` / `initial_lr`, which come from
the new config.  New groups without saved state start empty.  Without a mapping (old files) the
groups are taken positionally and only `lr` / `initial_lr` are overwritten.
"""
from __future__ import annotations

import copy


def remap_optimizer_state_dict(state_dict: dict, new_state_dict: dict, new_group_mapping: list[str],
                               optimizer_name: str) -> dict:
    sd = copy.copy(state_dict)
    new_groups = new_state_dict["param_groups"]
    if "param_group_mapping" not in sd:
        groups = [dict(g) for g in sd["param_groups"]]
        for g, ng in zip(groups, new_groups):
            g["lr"], g["initial_lr"] = ng["lr"], ng.get("initial_lr", ng["lr"])
        sd["param_groups"] = groups
        return sd
    old_state, old_groups = sd["state"], sd["param_groups"]
    old_mapping = list(sd["param_group_mapping"])
    old_opt = list(sd.get("param_group_optimizer_mapping", [optimizer_name] * len(old_mapping)))
    state, groups, idx = {}, [], 0
    for gi, name in enumerate(new_group_mapping):
        ng = new_groups[gi]
        if name in old_mapping and old_opt[old_mapping.index(name)] == optimizer_name:
            og = dict(old_groups[old_mapping.index(name)])
            params = []
            for old_i in og["params"]:
                if old_i in old_state:
                    state[idx] = old_state[old_i]
                params.append(idx)
                idx += 1
            og["params"] = params
            og["lr"], og["initial_lr"] = ng["lr"], ng.get("initial_lr", ng["lr"])
            groups.append(og)
        else:
            g = dict(ng)
            g["params"] = list(range(idx, idx + len(ng["params"])))
            idx += len(ng["params"])
            groups.append(g)
    sd["state"], sd["param_groups"] = state, groups
    return sd


def restore_training_state(model, config) -> None:
    """apply what a loader left on the model (InternalModelLoaderMixin.py:16-42): the optimizer state
    of a backup, remapped onto the groups setup_model just built."""
    sd = getattr(model, "optimizer_state_dict", None)
    if sd is not None and model.optimizer is not None:
        name = str(config.optimizer.optimizer)
        remapped = remap_optimizer_state_dict(sd, model.optimizer.state_dict(), model.param_group_mapping, name)
        model.optimizer.load_state_dict(remapped)
        model.optimizer_state_dict = None
