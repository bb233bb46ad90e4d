"""Record the reference's train-loop action timers (container only: imports /root/reference
read-only, stores data only).

    python tests/golden/make_timed_actions.py   -> tests/golden/timed_actions.json

Runs the reference's own modules/util/TimedActionMixin.py (repeating_action_needed,
single_action_elapsed) over a simulated progress of 3 epochs x 5 steps for every step / epoch /
NEVER / ALWAYS unit and a few intervals, with the combinations GenericTrainer uses for backups and
saves (GenericTrainer.py:506-516), and records the reference TrainConfig defaults of the backup /
save / output fields (TrainConfig.py:783-785, 981-989).  tests/test_host_logic.py replays the
same progress through onetrainer_amd/util/TimedActionMixin.py.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "timed_actions.json"
EPOCHS, STEPS = 3, 5
UNITS = ["STEP", "EPOCH", "NEVER", "ALWAYS"]
INTERVALS = [1, 2, 3]


def progress_sequence():
    seq = []
    g = 0
    for e in range(EPOCHS):
        for s in range(STEPS):
            seq.append((e, s, g))
            g += 1
    return seq


def main():
    sys.path.insert(0, str(REF))
    from modules.util.config.TrainConfig import TrainConfig
    from modules.util.enum.TimeUnit import TimeUnit
    from modules.util.TimedActionMixin import TimedActionMixin
    from modules.util.TrainProgress import TrainProgress

    cases = []
    for unit in UNITS:
        for interval in INTERVALS:
            for skip in (0, 2):
                m = TimedActionMixin()
                rec = {"unit": unit, "interval": interval, "skip": skip, "repeat0": [], "repeat1": [], "single": [],
                       "save": []}
                for e, s, g in progress_sequence():
                    tp = TrainProgress(epoch=e, epoch_step=s, global_step=g)
                    rec["repeat0"].append(m.repeating_action_needed("a", interval, TimeUnit(unit), tp, start_at_zero=False))
                    rec["repeat1"].append(m.repeating_action_needed("b", interval, TimeUnit(unit), tp, start_at_zero=True))
                    rec["single"].append(m.single_action_elapsed("c", skip, TimeUnit(unit), tp))
                    # GenericTrainer.__needs_save (GenericTrainer.py:511-516)
                    rec["save"].append(m.single_action_elapsed("d", skip, TimeUnit(unit), tp)
                                       and m.repeating_action_needed("e", interval, TimeUnit(unit), tp,
                                                                     start_at_zero=False))
                cases.append(rec)
    d = TrainConfig.default_values()
    defaults = {k: str(getattr(d, k)) if not isinstance(getattr(d, k), (int, float, bool)) else getattr(d, k)
                for k in ("backup_after", "backup_after_unit", "rolling_backup", "rolling_backup_count",
                          "backup_before_save", "save_every", "save_every_unit", "save_skip_first",
                          "save_filename_prefix", "output_dtype", "output_model_format", "output_model_destination")}
    OUT.write_text(json.dumps({"epochs": EPOCHS, "steps": STEPS, "cases": cases, "defaults": defaults}, indent=0))
    print(f"wrote {OUT} ({len(cases)} cases)")


if __name__ == "__main__":
    main()
