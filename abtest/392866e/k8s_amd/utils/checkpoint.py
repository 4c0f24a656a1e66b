"""TF-compatible checkpoint LAYOUT with a safetensors payload.

The reference leaves checkpoints to TensorFlow: files
``<job_dir>/model.ckpt-<step>.index`` / ``.data-00000-of-00001`` and a text
``checkpoint`` state file (``model_checkpoint_path: "model.ckpt-N"`` plus
``all_model_checkpoint_paths``), keep the last 5, write from the chief only,
restore on start. We keep exactly that naming, rotation and state file so
tooling that watches the job dir keeps working; the payload is ours:

* ``.data-00000-of-00001`` -- a safetensors file (fp32 master weights,
  optimizer state, extra buffers such as BN running stats), loadable with
  ``safetensors`` / ``torch.load``-free code paths only.
* ``.index`` -- JSON: format tag, step, tensor names/shapes/dtypes, metadata.

Writes are atomic (tmp + rename, state file last), so a retryable restart
(exit 128+) always finds a complete checkpoint.
"""
from __future__ import annotations

import json
import os
import re
import time
from typing import Dict, List, Optional, Tuple

import torch

STATE_FILE = "checkpoint"
PREFIX = "model.ckpt"
DATA_SUFFIX = ".data-00000-of-00001"


def _save_safetensors(tensors: Dict[str, torch.Tensor], path: str, metadata: Dict[str, str]):
    from safetensors.torch import save_file

    save_file({k: v.detach().contiguous().cpu() for k, v in tensors.items()}, path, metadata=metadata)


def _load_safetensors(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file

    return load_file(path)


def read_state(job_dir: str) -> Tuple[Optional[str], List[str]]:
    p = os.path.join(job_dir, STATE_FILE)
    if not os.path.exists(p):
        return None, []
    latest, allp = None, []
    for line in open(p):
        m = re.match(r'\s*(model_checkpoint_path|all_model_checkpoint_paths):\s*"(.*)"', line)
        if not m:
            continue
        if m.group(1) == "model_checkpoint_path":
            latest = m.group(2)
        else:
            allp.append(m.group(2))
    return latest, allp


def _write_state(job_dir: str, latest: str, allp: List[str]):
    tmp = os.path.join(job_dir, STATE_FILE + ".tmp")
    with open(tmp, "w") as f:
        f.write('model_checkpoint_path: "%s"\n' % latest)
        for p in allp:
            f.write('all_model_checkpoint_paths: "%s"\n' % p)
    os.replace(tmp, os.path.join(job_dir, STATE_FILE))


def save(job_dir: str, step: int, tensors: Dict[str, torch.Tensor], meta: Optional[dict] = None,
         keep: int = 5) -> str:
    os.makedirs(job_dir, exist_ok=True)
    name = "%s-%d" % (PREFIX, step)
    base = os.path.join(job_dir, name)
    md = {"format": "k8s_amd-safetensors-v1", "step": str(step), "time": str(time.time())}
    for k, v in (meta or {}).items():
        md[str(k)] = json.dumps(v) if not isinstance(v, str) else v
    _save_safetensors(tensors, base + DATA_SUFFIX + ".tmp", md)
    os.replace(base + DATA_SUFFIX + ".tmp", base + DATA_SUFFIX)
    index = {"format": md["format"], "step": step, "meta": meta or {},
             "tensors": {k: {"shape": list(v.shape), "dtype": str(v.dtype).replace("torch.", "")}
                         for k, v in tensors.items()}}
    with open(base + ".index.tmp", "w") as f:
        json.dump(index, f)
    os.replace(base + ".index.tmp", base + ".index")
    _, allp = read_state(job_dir)
    allp = [p for p in allp if p != name] + [name]
    for old in allp[:-keep] if keep > 0 else []:
        for suf in (".index", DATA_SUFFIX):
            try:
                os.remove(os.path.join(job_dir, old + suf))
            except FileNotFoundError:
                pass
    allp = allp[-keep:] if keep > 0 else allp
    _write_state(job_dir, name, allp)
    return base


def latest_checkpoint(job_dir: str) -> Optional[str]:
    latest, _ = read_state(job_dir)
    if latest and os.path.exists(os.path.join(job_dir, latest + ".index")):
        return os.path.join(job_dir, latest)
    return None


def load(base: str) -> Tuple[int, Dict[str, torch.Tensor], dict]:
    index = json.load(open(base + ".index"))
    tensors = _load_safetensors(base + DATA_SUFFIX)
    return int(index["step"]), tensors, index.get("meta", {})
