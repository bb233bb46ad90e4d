"""Reading a diffusers / transformers sub-module's weights from a local directory.

Restates the file resolution of modules/modelLoader/mixin/HFModelLoaderMixin.py:27-150 for local
paths (the hub download branch needs the network and is out of scope):
  * `<root>/<subfolder>/<shard_index_filename>` present -> sharded: every file named in its
    `weight_map` (sorted, de-duplicated) is read and merged;
  * otherwise the single `<model_filename>`;
  * any safetensors file missing -> the torch pickle `<pytorch_model_filename>` with
    `torch.load(weights_only=True)` (nothing executable is unpickled), unwrapping nested
    'state_dict' keys like the reference (line 113-115).
Keys the target module does not have are ignored by the caller (reference line 127-128).
"""
from __future__ import annotations

import json
import os

import torch
from safetensors.torch import load_file

DIFFUSERS_FILES = ("diffusion_pytorch_model.safetensors", "diffusion_pytorch_model.bin",
                   "diffusion_pytorch_model.safetensors.index.json")
TRANSFORMERS_FILES = ("model.safetensors", "pytorch_model.bin", "model.safetensors.index.json")


def read_sub_module_state_dict(root: str, subfolder: str | None, model_filename: str,
                               pytorch_model_filename: str | None, shard_index_filename: str) -> dict:
    base = os.path.join(root, subfolder) if subfolder else root
    if not os.path.isdir(base):
        raise FileNotFoundError(f"no such model directory: {base}")
    index = os.path.join(base, shard_index_filename)
    if os.path.isfile(index):
        with open(index) as f:
            names = sorted(set(json.load(f)["weight_map"].values()))
    else:
        names = [model_filename]
    files = [os.path.join(base, n) for n in names]
    sd: dict = {}
    if all(os.path.isfile(f) for f in files):
        for f in files:
            sd |= load_file(f)
        return sd
    if not pytorch_model_filename or not os.path.isfile(os.path.join(base, pytorch_model_filename)):
        raise FileNotFoundError(f"no weights in {base} ({', '.join(names)} / {pytorch_model_filename})")
    obj = torch.load(os.path.join(base, pytorch_model_filename), map_location="cpu", weights_only=True)
    while isinstance(obj, dict) and "state_dict" in obj:
        obj = obj["state_dict"]
    return dict(obj)


def read_diffusers_sub_module(root: str, subfolder: str | None) -> dict:
    return read_sub_module_state_dict(root, subfolder, *DIFFUSERS_FILES)


def read_single_file(path: str) -> dict:
    """a single-file checkpoint: .safetensors, or a torch pickle read with weights_only=True."""
    if not os.path.isfile(path):
        raise FileNotFoundError(path)
    if path.endswith(".safetensors"):
        return load_file(path)
    obj = torch.load(path, map_location="cpu", weights_only=True)
    while isinstance(obj, dict) and "state_dict" in obj:
        obj = obj["state_dict"]
    return dict(obj)
