"""The measured fused-LoRA tile table (onetrainer_amd/lora_plans_mi355x.json) and its lookup (kernels._lora_plan,
mirrored by ops_host.cpp lora_plan): well-formed entries, exact row counts first, and class entries applied only
while the tile grid fills its rounds of 256 CUs >= 85 % (the 832x1280 aspect buckets' 4160 / 16640 rows)."""
import json
import os

from onetrainer_amd import kernels as K

PATH = os.path.join(os.path.dirname(K.__file__), "lora_plans_mi355x.json")


def test_entries_well_formed():
    plans = json.load(open(PATH))["plans"]
    assert plans
    keys = set()
    for e in plans:
        assert e["form"] in (0, 1) and e["parts"] in (1, 3) and e["tile"] in (-1, 1, 4, 7, 8), e
        assert ("M" in e) != ("mclass" in e), e
        k = (e["form"], e["N"], e["K"], e["parts"], -e["M"] if "M" in e else e["mclass"])
        assert k not in keys, e
        keys.add(k)


def test_lookup_rules():
    # class entry at the measured rows: 128x160 for the level-2 1280-wide outputs (32 x 8 = 256 tiles)
    assert K._lora_plan(0, 1280, 1280, 1, 4096) == 7
    # ... at 4032 rows still one round (32 x 8), at 4160 rows 264 tiles: refused, the plan tile decides
    assert K._lora_plan(0, 1280, 1280, 1, 4032) == 7
    assert K._lora_plan(0, 1280, 1280, 1, 4160) is None
    # an exact-row entry wins over the class entry and is not fill-checked
    assert K._lora_plan(1, 1280, 3840, 3, 4160) == 1
    assert K._lora_plan(1, 1280, 3840, 3, 4096) == 7
    # two launches
    assert K._lora_plan(0, 10240, 1280, 1, 4096) == -1
    # no entry
    assert K._lora_plan(0, 320, 320, 1, 65536) is None


def test_native_lookup_matches_python():
    h = K._host()
    if h is None or not hasattr(h, "lora_plan"):
        import pytest
        pytest.skip("native host layer not built")
    for form in (0, 1):
        for N in (640, 1280, 1920, 2560, 3840, 5120, 10240):
            for Kd in (640, 1280, 1920, 2560, 3840, 5120, 10240):
                for parts in (1, 3):
                    for M in (4, 4032, 4096, 4160, 16128, 16384, 16640, 65536):
                        want = K._lora_plan(form, N, Kd, parts, M)
                        got = h.lora_plan(form, N, Kd, parts, M)
                        assert got == (0 if want is None else want), (form, N, Kd, parts, M)
