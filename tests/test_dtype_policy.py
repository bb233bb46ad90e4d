"""a20: the dtype policy (util/dtype_util.py) against the reference's own dtype decisions (CPU).

tests/golden/dtype_decisions.json holds, for TrainConfig.default_values() and the C1-C5 training presets (plus
dtype overrides), the reference's resolved per-part weight dtypes (TrainConfig.weight_dtypes()), its
create_autocast_context result as the setups call it and enable_grad_scaling (tests/golden/make_dtype_decisions.py,
run on the reference in the build container).  The build must (1) read the same decision from the same fields and
(2) take it, override it with a record, or refuse the config -- the pinned outcomes below.
"""
import json
import sys
from pathlib import Path
from types import SimpleNamespace

import pytest

from onetrainer_amd.util.dtype_util import dtype_plan, reference_decision, resolved_weight_dtypes

GOLD = Path(__file__).parent / "golden"
CASES = json.load(open(GOLD / "dtype_decisions.json"))["cases"]
REF = Path("/root/reference")


def stand_in(case):
    f = case["fields"]
    ns = SimpleNamespace(model_type=f["model_type"], training_method=f["training_method"], train_dtype=f["train_dtype"],
                         fallback_train_dtype=f["fallback_train_dtype"], weight_dtype=f["weight_dtype"],
                         lora_weight_dtype=f["lora_weight_dtype"])
    for p, wd in f["parts"].items():
        setattr(ns, p, SimpleNamespace(weight_dtype=wd))
    return ns


def case(source, **override):
    for c in CASES:
        if c["source"] == source and c["override"] == override:
            return c
    raise KeyError((source, override))


@pytest.mark.parametrize("i", range(len(CASES)))
def test_reads_the_reference_decision(i):
    c = CASES[i]
    cfg = stand_in(c)
    res = resolved_weight_dtypes(cfg)
    for k, v in c["resolved"].items():
        if k in res:
            assert res[k] == v, (k, res[k], v)
    ref = reference_decision(cfg)
    assert ref["compute"] == c["reference"]["compute"]
    assert ref["grad_scaler"] == c["reference"]["grad_scaler"]
    if c["reference"]["compute"] != "FLOAT_32":   # torch disables an fp32 autocast on the CPU the record ran on
        assert ref["autocast"] == c["reference"]["autocast"]


def _outcome(c):
    try:
        return sorted(o["field"] for o in dtype_plan(stand_in(c)).overrides)
    except ValueError:
        return "refused"


def test_pinned_outcomes():
    # TrainConfig.default_values() and C1's preset as it stands: SD 1.5 full fine-tune with fp32 master weights and a
    # FLOAT_16 train dtype -> fp32 masters (round 6), bf16 compute, no GradScaler, fp32 norm gradients rounded: recorded
    master = ["grad_scaler", "norm gradients", "train_dtype"]
    assert _outcome(case("default_values")) == master
    assert _outcome(case("sd15")) == master
    assert _outcome(case("sd15", train_dtype="BFLOAT_16")) == ["norm gradients"]
    assert dtype_plan(stand_in(case("sd15"))).master and dtype_plan(stand_in(case("sd15"))).network == "FLOAT_32"
    assert _outcome(case("sd15", train_dtype="FLOAT_32")) == "refused"   # fp32 compute is not built
    assert _outcome(case("sd15", train_dtype="BFLOAT_16", weight_dtype="BFLOAT_16")) == []   # C2
    # #sdxl 1.0.json: bf16 weights, train_dtype left at FLOAT_16 -> bf16 compute, recorded
    assert _outcome(case("sdxl")) == ["train_dtype"]
    assert _outcome(case("sdxl", train_dtype="BFLOAT_16")) == []
    assert _outcome(case("sdxl", train_dtype="FLOAT_32")) == "refused"
    # #sdxl 1.0 LoRA.json: fp16 frozen base, fp16 compute, fp32 adapters + GradScaler in the reference
    assert _outcome(case("sdxl_lora")) == ["grad_scaler", "train_dtype", "unet.weight_dtype"]
    assert _outcome(case("sdxl_lora", train_dtype="BFLOAT_16", weight_dtype="BFLOAT_16")) == []   # C4
    assert _outcome(case("sdxl_lora", lora_weight_dtype="BFLOAT_16")) == ["lora_weight_dtype", "train_dtype",
                                                                         "unet.weight_dtype"]
    # #flux LoRA.json: bf16 compute, NF4 transformer (bitsandbytes, CUDA-only) -> bf16 base, recorded (C5)
    assert _outcome(case("flux_lora")) == ["prior.weight_dtype"]


@pytest.mark.parametrize("i", range(len(CASES)))
def test_overrides_name_the_reference_values(i):
    c = CASES[i]
    try:
        plan = dtype_plan(stand_in(c))
    except ValueError as e:
        fine_tune = c["fields"]["training_method"] == "FINE_TUNE"
        net = c["resolved"]["prior" if c["fields"]["model_type"].startswith("FLUX") else "unet"]
        assert c["reference"]["compute"] == "FLOAT_32", (c, e)
        return
    fine_tune = c["fields"]["training_method"] == "FINE_TUNE"
    net = c["resolved"]["prior" if c["fields"]["model_type"].startswith("FLUX") else "unet"]
    assert plan.compute == "BFLOAT_16"
    assert plan.master == (fine_tune and net == "FLOAT_32")
    assert plan.network == ("FLOAT_32" if plan.master else "BFLOAT_16")
    for o in plan.overrides:
        if o["field"] == "train_dtype":
            assert o["reference"] == c["reference"]["compute"]
        elif o["field"].endswith(".weight_dtype"):
            assert o["reference"] == c["resolved"][o["field"].split(".")[0]]
        elif o["field"] == "lora_weight_dtype":
            assert o["reference"] == c["resolved"]["lora"]
        elif o["field"] == "grad_scaler":
            assert c["reference"]["grad_scaler"]
    assert ("grad_scaler" in [o["field"] for o in plan.overrides]) == c["reference"]["grad_scaler"]


def test_create_model_refuses_before_allocating():
    from onetrainer_amd.util import create
    with pytest.raises(ValueError, match="fp32 compute is not built"):
        create.create_model(stand_in(case("default_values", train_dtype="FLOAT_32")), "meta")


def test_fp32_master_store():
    """the reference's default (FLOAT_32 weights, full fine-tune): fp32 masters hold the trained values, the bf16
    working copy is their round-to-nearest cast (autocast's), the state dict / savers read the masters"""
    import torch

    from onetrainer_amd.module import unet as U
    from onetrainer_amd.util import create
    m = create.create_model(stand_in(case("default_values")), "cpu", seed=3, unet_config=U.tiny_sd15_config())
    st = m.unet.store
    assert st.master is not None and st.master.dtype == torch.float32 and st.data.dtype == torch.bfloat16
    assert st.grad.dtype == torch.bfloat16
    assert torch.equal(st.data, st.master.to(torch.bfloat16))
    sd = m.unet.state_dict()
    assert all(v.dtype == torch.float32 for v in sd.values())
    assert any(not torch.equal(v, v.bfloat16().float()) for v in sd.values())   # fp32 values, not bf16 ones
    # load -> fp32 master exactly, bf16 working copy re-cast
    m2 = create.create_model(stand_in(case("default_values")), "cpu", seed=9, unet_config=U.tiny_sd15_config())
    m2.unet.load_state_dict(sd)
    assert torch.equal(m2.unet.store.master, st.master) and torch.equal(m2.unet.store.data, st.data)
    # a bf16 network keeps no master copy and loads the same values as their bf16 cast
    m3 = create.create_model(stand_in(case("default_values", weight_dtype="BFLOAT_16")), "cpu", seed=9,
                             unet_config=U.tiny_sd15_config())
    assert m3.unet.store.master is None
    m3.unet.load_state_dict(sd)
    assert torch.equal(m3.unet.store.data, st.data)


def test_train_script_starts_from_the_reference_defaults(tmp_path):
    """scripts/train.py: a preset that leaves train_dtype unset gets the reference's FLOAT_16 (and the recorded bf16
    override), not this build's own default"""
    import importlib.util
    spec = importlib.util.spec_from_file_location("train_script", Path(__file__).parents[1] / "scripts" / "train.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    p = tmp_path / "c.json"
    p.write_text(json.dumps({"model_type": "STABLE_DIFFUSION_XL_10_BASE", "weight_dtype": "BFLOAT_16",
                             "vae": {"weight_dtype": "FLOAT_32"}}))
    cfg = mod.load_config(str(p))
    assert cfg.train_dtype == "FLOAT_16"
    assert [o["field"] for o in dtype_plan(cfg).overrides] == ["train_dtype"]
    p.write_text(json.dumps({"model_type": "STABLE_DIFFUSION_15"}))   # the reference's defaults: fp32 weights
    plan = dtype_plan(mod.load_config(str(p)))
    assert plan.master and [o["field"] for o in plan.overrides] == ["train_dtype", "norm gradients", "grad_scaler"]


@pytest.mark.skipif(not REF.exists(), reason="reference checkout only in the build container")
@pytest.mark.parametrize("preset", ["#sd 1.5.json", "#sdxl 1.0.json", "#sdxl 1.0 LoRA.json", "#flux LoRA.json"])
def test_real_reference_trainconfig(preset):
    """the plan taken on the reference's own enum-typed TrainConfig object equals the one taken on the record"""
    sys.path.insert(0, str(REF))
    from modules.util.config.TrainConfig import TrainConfig
    c = TrainConfig.default_values()
    with open(REF / "training_presets" / preset) as f:
        c.from_dict(json.load(f))
    key = {"#sd 1.5.json": "sd15", "#sdxl 1.0.json": "sdxl", "#sdxl 1.0 LoRA.json": "sdxl_lora",
           "#flux LoRA.json": "flux_lora"}[preset]
    rec = case(key)
    try:
        got = sorted(o["field"] for o in dtype_plan(c).overrides)
    except ValueError:
        got = "refused"
    assert got == _outcome(rec)
