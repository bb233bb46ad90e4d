"""The plugin boundary on the reference's enum-typed TrainConfig (CPU).

The reference's GenericTrainer hands its own TrainConfig -- Enum members in every enum field
(modules/util/enum/LossScaler.py, TimestepDistribution.py, Optimizer.py ...) -- to
predict / calculate_loss / setup_model.  tests/golden/config_decisions.json holds, for the C1-C5
presets and every LossScaler / LossWeight / TimestepDistribution override, the field values and
the per-sample losses the reference's own ModelSetupDiffusionLossMixin computed with that config
(tests/golden/make_config_decisions.py).  Here an enum-typed stand-in is rebuilt from those
strings, and the plugin's decisions (loss_plan / timestep_plan / optimizer) driven through
oracle.diffusion must reproduce the reference's losses.  When /root/reference is present (the
build container) the same decisions are also taken on the reference's real TrainConfig objects.
"""
import json
import sys
from enum import Enum
from pathlib import Path
from types import SimpleNamespace

import pytest
import torch

from oracle import diffusion as OD
from onetrainer_amd.modelSetup.BaseStableDiffusionXLSetup import LOSS_FN, loss_plan, timestep_plan
from onetrainer_amd.util.config.plain import PlainConfig, plain

GOLD = Path(__file__).parent / "golden"
CASES = json.load(open(GOLD / "config_decisions.json"))["cases"]
REF = Path("/root/reference")
NAME_OF = {v: k for k, v in LOSS_FN.items()}


def _enum(cls_name, val):
    return Enum(cls_name, {val: val})[val]


def stand_in(case):
    ns = SimpleNamespace(**case["num_fields"])
    for k, v in case["enum_fields"].items():
        setattr(ns, k, _enum(k, v))
    ns.optimizer = SimpleNamespace(optimizer=_enum("Optimizer", case["optimizer"]))
    return ns


def inputs():
    sys.path.insert(0, str(GOLD))
    from make_config_decisions import inputs as mk
    return mk()


def oracle_losses(plan, case):
    pred, target, lw, t = inputs()
    if case["flow"]:
        return OD.flow_matching_losses(pred, target, lw, t, "SIGMA" if plan["loss_fn"] == 4 else "CONSTANT",
                                       mse_strength=plan["mse_strength"], batch_size_scale=plan["batch_size_scale"],
                                       ga_scale=plan["ga_scale"])
    return OD.diffusion_losses(pred, target, lw, t, OD.scaled_linear_betas(), NAME_OF[plan["loss_fn"]],
                               gamma=plan["gamma"], v_pred=case["v_pred"], mse_strength=plan["mse_strength"],
                               batch_size_scale=plan["batch_size_scale"], ga_scale=plan["ga_scale"])


@pytest.mark.parametrize("i", range(len(CASES)))
def test_enum_config_decisions_reproduce_reference_losses(i):
    case = CASES[i]
    cfg = plain(stand_in(case))
    assert isinstance(cfg.loss_scaler, str) and isinstance(cfg.optimizer, PlainConfig)
    plan = loss_plan(cfg, flow=case["flow"])
    torch.testing.assert_close(oracle_losses(plan, case), torch.tensor(case["reference_losses"]), rtol=1e-6, atol=0)
    assert timestep_plan(cfg) == {"UNIFORM": 0, "LOGIT_NORMAL": 1}[case["enum_fields"]["timestep_distribution"]]
    assert cfg.optimizer.optimizer == "ADAMW"


def test_plain_passes_strings_and_writes_through():
    ns = SimpleNamespace(loss_scaler="BATCH", batch_size=2, part=None)
    p = plain(ns)
    assert p.loss_scaler == "BATCH" and plain(p) is p
    p.batch_size = 5
    assert ns.batch_size == 5
    assert p.dp_bucket_mb == 256 and p.dp_reduce_fp32 is False   # build-only defaults


@pytest.mark.skipif(not REF.exists(), reason="reference checkout only in the build container")
@pytest.mark.parametrize("preset", ["#sd 1.5.json", "#sdxl 1.0.json", "#sdxl 1.0 LoRA.json", "#flux LoRA.json"])
def test_real_reference_trainconfig(preset):
    """the reference's TrainConfig object itself (enum members), loaded from its preset JSON."""
    sys.path.insert(0, str(REF))
    from modules.util.config.TrainConfig import TrainConfig
    from modules.util.enum.LossScaler import LossScaler
    c = TrainConfig.default_values()
    with open(REF / "training_presets" / preset) as f:
        c.from_dict(json.load(f))
    p = plain(c)
    assert p.model_type == c.model_type.value and p.optimizer.optimizer == "ADAMW"
    assert p.text_encoder.train in (True, False) and p.text_encoder.dropout_probability == c.text_encoder.dropout_probability
    for s in LossScaler:
        c.loss_scaler, c.batch_size, c.gradient_accumulation_steps = s, 4, 3
        plan = loss_plan(plain(c), flow="flux" in preset)
        want_bs = 1 if s in (LossScaler.NONE, LossScaler.GRADIENT_ACCUMULATION) else 4
        want_ga = 1 if s in (LossScaler.NONE, LossScaler.BATCH) else 3
        assert (plan["batch_size_scale"], plan["ga_scale"]) == (want_bs, want_ga)
