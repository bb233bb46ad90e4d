#!/usr/bin/env python3
"""Command-line training entry: the reference's scripts/train.py:15-43 on this build.

    python scripts/train.py --config-path config.json [--secrets-path s.json]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        scripts/train.py --config-path config.json          # data parallel, one rank per GPU

Same flow as the reference: TrainConfig.default_values().from_dict(json) ->
GenericTrainer(config, callbacks, commands) -> start() -> train() -> end() (end also after a
KeyboardInterrupt when backup_before_save is set).  The config is the reference's own JSON
(training presets, UI-saved configs); fields this build does not read are kept and ignored.
The arguments of modules/util/args/TrainArgs.py:15-29 are accepted; --callback-path /
--command-path (UI pickle pipes, CloudTrainer) are accepted and unused.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class TrainCallbacks:
    """modules/util/callbacks/TrainCallbacks.py surface (no UI here)."""

    def on_update_status(self, status: str):
        print(status, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="One Trainer (MI355X build) training script")
    ap.add_argument("--config-path", type=str, required=True, dest="config_path")
    ap.add_argument("--secrets-path", type=str, default=None, dest="secrets_path")
    ap.add_argument("--callback-path", type=str, default=None, dest="callback_path")
    ap.add_argument("--command-path", type=str, default=None, dest="command_path")
    ap.add_argument("--max-steps", type=int, default=None, help="(build-only) stop after this many steps")
    return ap.parse_args(argv)


def load_config(path: str):
    """TrainConfig.default_values().from_dict(json) as scripts/train.py:23-25 does, from the reference's defaults
    (TrainConfig.reference_defaults): fields a JSON leaves unset take the reference's values, and the dtype policy
    (util/dtype_util.dtype_plan) records or refuses what this build does with them"""
    from onetrainer_amd.util.config.TrainConfig import TrainConfig
    train_config = TrainConfig.reference_defaults()
    with open(path, "r") as f:
        train_config.from_dict(json.load(f))
    return train_config


def main(argv=None):
    args = parse_args(argv)
    from onetrainer_amd.trainer.GenericTrainer import GenericTrainer
    from onetrainer_amd.util.TrainCommands import TrainCommands

    callbacks = TrainCallbacks()
    commands = TrainCommands()
    train_config = load_config(args.config_path)
    try:   # secrets (hub tokens, cloud keys) are not used by this build; a named file must exist
        with open("secrets.json" if args.secrets_path is None else args.secrets_path, "r") as f:
            train_config.extra["secrets"] = json.load(f)
    except FileNotFoundError:
        if args.secrets_path is not None:
            raise

    trainer = GenericTrainer(train_config, callbacks, commands)
    trainer.start()
    canceled = False
    try:
        trainer.train(max_steps=args.max_steps)
    except KeyboardInterrupt:
        canceled = True
    if not canceled or train_config.backup_before_save:   # scripts/train.py:36-43
        trainer.end()
    return trainer


if __name__ == "__main__":
    main()
