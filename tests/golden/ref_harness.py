"""Import harness for the reference's own setup / trainer code in THIS container (SURVEY.md
Appendix A).  Test-fixture tooling only: used by tests/golden/make_golden_glue.py, never at test
or run time, never on the GPU box.

diffusers, mgds, tensorboard, torchvision, cv2, customtkinter, scalene, bitsandbytes and
omi_model_standards are not installable offline; a meta-path finder hands out empty stand-in
packages for them so that the reference's modules import.  Attribute access on a stand-in returns
a dummy class (dunder lookups raise AttributeError so `inspect` inside torch keeps working).
transformers is imported first (its torchvision probes must see the real environment), and its
`Trie` is re-exported where transformers 4.x had it (the reference pins 4.48.3).
"""
from __future__ import annotations

import importlib.abc
import importlib.machinery
import sys
import types

REF = "/root/reference"
STUB_PREFIXES = ("diffusers", "mgds", "torch.utils.tensorboard", "tensorboard", "torchvision", "cv2",
                 "customtkinter", "scalene", "bitsandbytes", "omi_model_standards")


class _Dummy:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Dummy()

    def __getattr__(self, k):
        if k.startswith("__"):
            raise AttributeError(k)
        return _Dummy


class _StubModule(types.ModuleType):
    def __getattr__(self, k):
        if k.startswith("__"):
            raise AttributeError(k)
        cls = type(k, (_Dummy,), {})
        setattr(self, k, cls)
        return cls


class _StubFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, name, path, target=None):
        if any(name == p or name.startswith(p + ".") for p in STUB_PREFIXES):
            return importlib.machinery.ModuleSpec(name, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _StubModule(spec.name)
        m.__path__ = []
        return m

    def exec_module(self, module):
        pass


_installed = False


def install():
    global _installed
    if _installed:
        return
    import transformers  # (before the finder: its availability probes must be real)
    import transformers.tokenization_python as tp
    # transformers 5 serves `transformers.tokenization_utils` as a lazy alias of
    # tokenization_utils_sentencepiece; give that target the 4.x name the reference imports
    import transformers.tokenization_utils_sentencepiece as tus
    if not hasattr(tus, "Trie"):
        tus.Trie = tp.Trie
    sys.meta_path.insert(0, _StubFinder())
    if REF not in sys.path:
        sys.path.insert(0, REF)
    # import order of scripts/train.py:7 (GenericTrainer first: optimizer_util <-> create cycle)
    import modules.trainer.GenericTrainer  # noqa: F401
    _installed = True
