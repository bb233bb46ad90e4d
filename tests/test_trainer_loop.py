"""The train loop around the step (CPU): action timers pinned to the reference's own
TimedActionMixin (tests/golden/timed_actions.json), backup / save commands executed at
optimizer-update boundaries (GenericTrainer.py:653-668), stop, end() (GenericTrainer.py:766-806).
train_step / backup / save / the model writer are replaced by recorders: no GPU, no model."""
import json
from pathlib import Path
from types import SimpleNamespace

import pytest
import torch

from onetrainer_amd.trainer import GenericTrainer as GT
from onetrainer_amd.util.config.TrainConfig import TrainConfig
from onetrainer_amd.util.TimedActionMixin import TimedActionMixin
from onetrainer_amd.util.TrainCommands import TrainCommands
from onetrainer_amd.util.TrainProgress import TrainProgress

FIX = json.loads((Path(__file__).parent / "golden" / "timed_actions.json").read_text())


@pytest.mark.parametrize("case", FIX["cases"], ids=lambda c: f"{c['unit']}-{c['interval']}-{c['skip']}")
def test_timers_match_reference(case):
    m = TimedActionMixin()
    got = {"repeat0": [], "repeat1": [], "single": [], "save": []}
    for e in range(FIX["epochs"]):
        for s in range(FIX["steps"]):
            tp = TrainProgress(epoch=e, epoch_step=s, global_step=e * FIX["steps"] + s)
            u, n, k = case["unit"], case["interval"], case["skip"]
            got["repeat0"].append(m.repeating_action_needed("a", n, u, tp, start_at_zero=False))
            got["repeat1"].append(m.repeating_action_needed("b", n, u, tp, start_at_zero=True))
            got["single"].append(m.single_action_elapsed("c", k, u, tp))
            got["save"].append(m.single_action_elapsed("d", k, u, tp)
                               and m.repeating_action_needed("e", n, u, tp, start_at_zero=False))
    for key in got:
        assert got[key] == case[key], key


def test_wallclock_timer_starts_at_first_query(monkeypatch):
    import onetrainer_amd.util.TimedActionMixin as TM
    now = [1000.0]
    monkeypatch.setattr(TM.time, "time", lambda: now[0])
    m = TimedActionMixin()
    tp = TrainProgress()
    assert not m.repeating_action_needed("b", 1, "MINUTE", tp, start_at_zero=False)
    now[0] += 59
    assert not m.repeating_action_needed("b", 1, "MINUTE", tp, start_at_zero=False)
    now[0] += 2
    assert m.repeating_action_needed("b", 1, "MINUTE", tp, start_at_zero=False)
    assert not m.repeating_action_needed("b", 1, "MINUTE", tp, start_at_zero=False)
    assert m.repeating_action_needed("z", 1, "MINUTE", tp, start_at_zero=True)   # fires at once


def test_config_defaults_match_reference():
    d = TrainConfig.default_values()
    for k, v in FIX["defaults"].items():
        assert getattr(d, k) == v, k


@pytest.fixture(autouse=True)
def _in_tmp(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)   # train() opens its scalar log under the (relative) workspace_dir


class _Loader:
    def __init__(self, n):
        self.n = n

    def get_data_set(self):
        return SimpleNamespace(start_next_epoch=lambda: None, approximate_length=lambda: self.n)

    def get_data_loader(self):
        return iter(range(self.n))


def _trainer(ga=1, epochs=2, steps=6, **cfg_kw):
    cfg = TrainConfig.default_values()
    cfg.gradient_accumulation_steps = ga
    cfg.epochs = epochs
    for k, v in cfg_kw.items():
        setattr(cfg, k, v)
    tp = TrainProgress()
    tr = GT.GenericTrainer(cfg, model=SimpleNamespace(train_progress=tp), data_loader=_Loader(steps))
    log = []

    def step(batch):   # the loop-visible effects of GenericTrainer.train_step
        update = tr._is_update_step(tp)
        log.append(("step", tp.global_step))
        if update:
            tr.model_setup.report_to_tensorboard(None, cfg, tr.lr_scheduler, tr.tensorboard)
            tr.one_step_trained = True
        tr._has_gradient = not update
        tp.next_step(cfg.batch_size)
        return torch.zeros(())

    tr.train_step = step
    tr.model_setup = SimpleNamespace(report_to_tensorboard=lambda m, c, sch, tb: log.append(("report", tp.global_step)))
    tr.lr_scheduler = SimpleNamespace(get_last_lr=lambda: [1e-4])
    tr.backup = lambda t=None: log.append(("backup", tp.global_step))
    tr.save = lambda t=None: log.append(("save", tp.global_step))
    return tr, log


def _actions(log, kind):
    return [g for k, g in log if k == kind]


def test_backup_every_two_steps():
    tr, log = _trainer(backup_after=2, backup_after_unit="STEP")
    tr.train(log_every=0)
    # GenericTrainer.__needs_backup fires when (global_step + 1) % 2 == 0 and runs before that step
    assert _actions(log, "backup") == [1, 3, 5, 7, 9, 11]
    assert _actions(log, "save") == []


def test_commands_wait_for_the_update_boundary():
    """with GA=2 a backup raised on a micro-step with a gradient pending runs before the next
    update-cycle's first micro-step (GenericTrainer.py:653-668 `if not has_gradient`)."""
    tr, log = _trainer(ga=2, backup_after=2, backup_after_unit="STEP")
    tr.train(log_every=0)
    assert _actions(log, "backup") == [2, 4, 6, 8, 10]


def test_save_every_epoch_after_skip():
    tr, log = _trainer(epochs=3, steps=4, save_every=1, save_every_unit="EPOCH", save_skip_first=1)
    tr.train(log_every=0)
    # epoch-unit saves fire at the first step of each epoch after the first (start_at_zero=False), and
    # save_skip_first=1 EPOCH skips none of those (epoch + 1 > 1 from epoch 1 on)
    assert _actions(log, "save") == [4, 8]


def test_external_commands_and_stop():
    cmds = TrainCommands()
    tr, log = _trainer(steps=10, backup_after_unit="NEVER")
    tr.commands = cmds
    orig = tr.train_step

    def step(batch):
        g = tr.model.train_progress.global_step
        if g == 2:
            cmds.save()
        if g == 5:
            cmds.stop()
        return orig(batch)

    tr.train_step = step
    tr.train(log_every=0)
    assert _actions(log, "save") == [3]
    assert _actions(log, "step")[-1] == 5     # stop is honoured right after the step that raised it
    assert not cmds.get_and_reset_save_command()


def test_gc_restored_after_an_exception():
    import gc
    tr, log = _trainer(steps=5)
    orig = tr.train_step

    def step(batch):
        if tr.model.train_progress.global_step == 3:
            raise KeyboardInterrupt
        return orig(batch)

    tr.train_step = step
    with pytest.raises(KeyboardInterrupt):
        tr.train(log_every=0)
    assert gc.isenabled()
    assert gc.get_freeze_count() == 0


def test_end_backs_up_then_saves(tmp_path):
    tr, log = _trainer(steps=2, output_model_destination=str(tmp_path), output_model_format="SAFETENSORS",
                       save_filename_prefix="run-", output_dtype="BFLOAT_16")
    written = []
    tr._write_model = lambda path, fmt: written.append((path, fmt, tr.config.output_dtype)) or path
    assert tr.end() is None and written == []          # nothing trained: nothing saved (GenericTrainer.py:767)
    tr.train(log_every=0)
    tr.end()
    assert _actions(log, "backup") == [4]             # backup_before_save (default True)
    (path, fmt, dt), = written
    assert fmt == "SAFETENSORS" and dt == "BFLOAT_16"
    assert Path(path).parent == tmp_path and Path(path).name.startswith("run-") and path.endswith(".safetensors")
    assert GT._torch_dtype("BFLOAT_16") is torch.bfloat16 and GT._torch_dtype("FLOAT_32") is torch.float32


def test_end_without_backup_to_a_file(tmp_path):
    dest = str(tmp_path / "out" / "model.safetensors")
    tr, log = _trainer(steps=1, output_model_destination=dest, backup_before_save=False)
    written = []
    tr._write_model = lambda path, fmt: written.append(path) or path
    tr.train(log_every=0)
    tr.end()
    assert written == [dest] and _actions(log, "backup") == []


def test_loss_and_smooth_loss_scalars():
    """GenericTrainer.py:719-732: per update step `loss/train_step` = the sum of its micro-step losses and
    `smooth_loss/train_step` = EMA with decay min(0.99, 1 - 1/k), at the update micro-step's global_step;
    report_to_tensorboard once per update step"""
    from onetrainer_amd.util.tensorboard import read_scalars
    tr, log = _trainer(ga=2, epochs=1, steps=6)
    tp = tr.model.train_progress
    orig = tr.train_step

    def step(batch):
        v = float(tp.global_step)
        orig(batch)
        return torch.tensor(v)

    tr.train_step = step
    tr.train(log_every=4)
    assert _actions(log, "report") == [1, 3, 5]          # at the update step, before next_step()
    rows = read_scalars(tr.tensorboard.log_dir)
    loss = [(r["step"], r["value"]) for r in rows if r["tag"] == "loss/train_step"]
    smooth = [(r["step"], r["value"]) for r in rows if r["tag"] == "smooth_loss/train_step"]
    assert loss == [(1, 1.0), (3, 5.0), (5, 9.0)]
    assert [st for st, _ in smooth] == [1, 3, 5] and [v for _, v in smooth] == pytest.approx([1.0, 3.0, 5.0])
    tr.end()


def test_report_learning_rates():
    """BaseModelSetup.report_to_tensorboard (BaseModelSetup.py:96-119): lr/<display-name prefix>, first group wins"""
    from onetrainer_amd.modelSetup.BaseStableDiffusionXLSetup import report_learning_rates
    from onetrainer_amd.util.NamedParameterGroup import NamedParameterGroup, NamedParameterGroupCollection
    pgc = NamedParameterGroupCollection()
    for name in ("unet", "te/1", "te/2"):
        pgc.add_group(NamedParameterGroup(name, [], 1.0, display_name=name))
    got = []
    tb = SimpleNamespace(add_scalar=lambda tag, v, step: got.append((tag, v, step)))
    model = SimpleNamespace(parameters=pgc, train_progress=SimpleNamespace(global_step=7))
    report_learning_rates(model, SimpleNamespace(get_last_lr=lambda: [1.0, 2.0, 3.0]), tb)
    assert got == [("lr/unet", 1.0, 7), ("lr/te", 2.0, 7)]


@pytest.mark.parametrize("scaler,factor", [("NONE", 1.0), ("BATCH", 2.0), ("GRADIENT_ACCUMULATION", 2 ** 0.5),
                                           ("BOTH", 8 ** 0.5)])
def test_learning_rate_scaler(scaler, factor):
    """NamedParameterGroup.py:36-60: lr x sqrt(batch_size x GA) as learning_rate_scaler selects"""
    from onetrainer_amd.util.NamedParameterGroup import NamedParameterGroup, NamedParameterGroupCollection
    cfg = TrainConfig.default_values()
    cfg.batch_size, cfg.gradient_accumulation_steps, cfg.learning_rate_scaler = 4, 2, scaler
    pgc = NamedParameterGroupCollection()
    pgc.add_group(NamedParameterGroup("unet", [], None))
    pgc.add_group(NamedParameterGroup("te", [], 1e-5))
    g = pgc.parameters_for_optimizer(cfg)
    assert g[0]["lr"] == pytest.approx(cfg.learning_rate * factor) and g[0]["initial_lr"] == g[0]["lr"]
    assert g[1]["lr"] == pytest.approx(1e-5 * factor)


class _FakeSetup:
    """predict / calculate_loss / report hooks of a model setup over one scalar parameter (no GPU)"""

    def __init__(self, tb_log):
        self.tb_log = tb_log

    def predict(self, model, batch, cfg, tp):
        return {"p": model.w * 2.0}

    def calculate_loss(self, model, batch, out, cfg):
        return (out["p"] ** 2).sum()

    def report_to_tensorboard(self, model, cfg, sch, tb):
        from onetrainer_amd.modelSetup.BaseStableDiffusionXLSetup import report_learning_rates
        report_learning_rates(model, sch, tb)

    def after_optimizer_step(self, model, cfg, tp):
        pass


def _real_step_trainer(ga):
    from onetrainer_amd.util.NamedParameterGroup import NamedParameterGroup, NamedParameterGroupCollection
    cfg = TrainConfig.default_values()
    cfg.gradient_accumulation_steps = ga
    cfg.clip_grad_norm = None
    tp = TrainProgress()
    w = torch.nn.Parameter(torch.ones(()))
    pgc = NamedParameterGroupCollection()
    pgc.add_group(NamedParameterGroup("unet", [w], 1.0, display_name="unet"))
    opt = torch.optim.SGD([w], lr=0.1)
    store = SimpleNamespace(begin_backward=lambda: None, finish_backward=lambda: None, accumulating=False)
    model = SimpleNamespace(w=w, optimizer=opt, train_progress=tp, train_store=store, parameters=pgc)
    got = []
    tr = GT.GenericTrainer(cfg, model=model, model_setup=_FakeSetup(got))
    tr.lr_scheduler = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0)
    tr.tensorboard = SimpleNamespace(add_scalar=lambda tag, v, st: got.append((tag, st)))
    return tr, got


def test_train_step_reports_lr_at_the_update_step():
    """BaseModelSetup.report_to_tensorboard runs inside the update branch before train_progress.next_step
    (GenericTrainer.py:720-754): lr/<group> carries the update step's own global_step, not the next one"""
    tr, got = _real_step_trainer(ga=2)
    for _ in range(4):
        tr.train_step({})
    assert got == [("lr/unet", 1), ("lr/unet", 3)]


def test_one_step_trained_only_after_an_update():
    """GenericTrainer.py:749: a micro-step without an optimizer update does not count as trained, so end()
    after a stop inside the first accumulation window saves nothing"""
    tr, _ = _real_step_trainer(ga=2)
    tr.train_step({})
    assert not tr.one_step_trained
    tr.train_step({})
    assert tr.one_step_trained


def test_losses_flushed_without_log_every():
    """train(log_every=0): the loss scalars are still written (every 32 steps and at the end) and the
    device loss history stays bounded"""
    from onetrainer_amd.util.tensorboard import read_scalars
    tr, log = _trainer(epochs=1, steps=70)
    tp = tr.model.train_progress
    orig = tr.train_step

    def step(batch):
        v = float(tp.global_step)
        orig(batch)
        return torch.tensor(v)

    tr.train_step = step
    tr.train(log_every=0)
    rows = read_scalars(tr.tensorboard.log_dir)
    loss = [(r["step"], r["value"]) for r in rows if r["tag"] == "loss/train_step"]
    assert loss == [(g, float(g)) for g in range(70)]
    assert len(tr.loss_history) <= 32 and not tr._update_losses
    tr.end()
