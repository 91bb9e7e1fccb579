"""Checkpoint / resume for the training state (reference: utils/pipeline.py:38-48
tf.train.Checkpoint(transformer, optimizer) + CheckpointManager(max_to_keep=100),
restored at construction when a checkpoint exists; train.py:37-41,94-96).

The reference writes TF's own checkpoint format, which nothing here can read
(TensorFlow is not installed). This build writes one safetensors file per
checkpoint holding
  model/<state_dict key>           every parameter and buffer (fp32 masters,
                                   Keras layouts, frozen-BN statistics)
  optimizer/{m,v,vhat}/<param>     the AMSGrad slots of every trainable tensor
  optimizer/iterations             Keras `iterations` (int64, drives the lr
                                   schedule and the bias correction)
keyed by parameter NAME, so a checkpoint restores into any arena ordering.
A small JSON index (`checkpoint`) in the directory lists the files, newest
last, like TF's `checkpoint` state file.

Only rank 0 writes under torch.distributed (the ranks hold identical
replicas after every all-reduced step: the parameters through the gradient
all-reduce, the MobileNetV2 BatchNorm moving statistics because the
data-parallel engine makes those layers cross-replica, fpnmt.dist.
set_sync_batchnorm); every rank restores.
"""
from __future__ import annotations

import json
import os

import torch
import torch.distributed as dist

FORMAT = "fpnmt-ckpt-v1"


def _is_writer():
    return not dist.is_initialized() or dist.get_rank() == 0


class Checkpoint:
    """tf.train.Checkpoint(transformer=..., optimizer=...): `optimizer` is the
    fpnmt.train.TrainEngine that owns the parameter arena (or None to save the
    model alone)."""

    def __init__(self, transformer, optimizer=None):
        self.transformer = transformer
        self.optimizer = optimizer
        self.save_counter = 0

    # ------------------------------------------------------------ tensors
    def state_tensors(self):
        out = {}
        for k, v in self.transformer.state_dict().items():
            out["model/" + k] = v.detach().to("cpu", copy=True).contiguous()
        eng = self.optimizer
        if eng is not None:
            a = eng.arena
            for name, p, off in zip(a.names, a.params, a.offsets):
                n = p.numel()
                for slot, buf in (("m", a.m), ("v", a.v), ("vhat", a.vhat)):
                    out[f"optimizer/{slot}/{name}"] = buf[off:off + n].view(p.shape).detach().cpu().clone()
            out["optimizer/iterations"] = a.step.detach().cpu().clone()
        return out

    def write(self, path):
        from safetensors.torch import save_file
        self.save_counter += 1
        if _is_writer():
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            tmp = path + ".tmp"
            save_file(self.state_tensors(), tmp, metadata={"format": FORMAT, "save_counter": str(self.save_counter)})
            os.replace(tmp, path)
        if dist.is_initialized():
            dist.barrier()
        return path

    @torch.no_grad()
    def restore(self, path):
        """Load every tensor back in place (parameters stay arena views, so
        captured hipGraphs remain valid) and mark the compute copies stale."""
        from safetensors import safe_open
        from . import layers as flayers
        with safe_open(path, framework="pt") as f:
            meta = f.metadata() or {}
            if meta.get("format") != FORMAT:
                raise ValueError(f"{path}: not an fpnmt checkpoint (format {meta.get('format')!r})")
            keys = set(f.keys())
            sd = self.transformer.state_dict()
            missing = [k for k in sd if "model/" + k not in keys]
            if missing:
                raise KeyError(f"{path}: checkpoint lacks {len(missing)} model tensors, e.g. {missing[:3]}")
            for k, v in sd.items():
                t = f.get_tensor("model/" + k)
                if tuple(t.shape) != tuple(v.shape):
                    raise ValueError(f"{path}: {k} has shape {tuple(t.shape)}, model expects {tuple(v.shape)}")
                v.copy_(t.to(v.dtype))
            eng = self.optimizer
            if eng is not None and "optimizer/iterations" in keys:
                a = eng.arena
                for name, p, off in zip(a.names, a.params, a.offsets):
                    n = p.numel()
                    for slot, buf in (("m", a.m), ("v", a.v), ("vhat", a.vhat)):
                        buf[off:off + n].copy_(f.get_tensor(f"optimizer/{slot}/{name}").reshape(-1))
                a.step.copy_(f.get_tensor("optimizer/iterations"))
            self.save_counter = int(meta.get("save_counter", self.save_counter))
        for m in self.transformer.modules():  # frozen-BN folds read the restored statistics
            if hasattr(m, "refresh_bn") and getattr(m, "bn_scale", None) is not None:
                m.refresh_bn()
        flayers.invalidate_weights()
        if any(p.is_cuda for p in self.transformer.parameters()):
            flayers.prepare_all(self.transformer)
        return self


class CheckpointManager:
    """tf.train.CheckpointManager(ckpt, directory, max_to_keep): numbered
    `ckpt-<n>.safetensors` files, the oldest deleted past max_to_keep."""

    INDEX = "checkpoint"

    def __init__(self, checkpoint, directory, max_to_keep=5):
        self.checkpoint = checkpoint
        self.directory = directory
        self.max_to_keep = max_to_keep
        self.checkpoints = self._read_index()
        if self.checkpoints:
            n = os.path.basename(self.checkpoints[-1]).split("-")[-1].split(".")[0]
            checkpoint.save_counter = max(checkpoint.save_counter, int(n))

    def _index_path(self):
        return os.path.join(self.directory, self.INDEX)

    def _read_index(self):
        try:
            with open(self._index_path()) as f:
                names = json.load(f)["all_model_checkpoint_paths"]
        except (OSError, ValueError, KeyError):
            return []
        return [os.path.join(self.directory, n) for n in names if os.path.exists(os.path.join(self.directory, n))]

    @property
    def latest_checkpoint(self):
        return self.checkpoints[-1] if self.checkpoints else None

    def save(self):
        n = self.checkpoint.save_counter + 1
        path = os.path.join(self.directory, f"ckpt-{n}.safetensors")
        self.checkpoint.write(path)
        self.checkpoints.append(path)
        while self.max_to_keep is not None and len(self.checkpoints) > self.max_to_keep:
            old = self.checkpoints.pop(0)
            if _is_writer() and os.path.exists(old):
                os.remove(old)
        if _is_writer():
            with open(self._index_path(), "w") as f:
                json.dump({"model_checkpoint_path": os.path.basename(path),
                           "all_model_checkpoint_paths": [os.path.basename(p) for p in self.checkpoints]}, f)
        return path
