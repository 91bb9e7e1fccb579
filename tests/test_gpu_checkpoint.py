"""Checkpoint / resume on the GPU (utils/pipeline.py:38-48 restore at
construction, train.py:36-41 resume, :94-96 save_weights): the bf16
hipGraph-replayed training step is bitwise deterministic, so a run that is
checkpointed after k steps and resumed must reproduce the uninterrupted run
exactly — losses and the whole parameter / AMSGrad state."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pipeline(ckpt_dir):
    from fpnmt.layers import Init
    from utils.pipeline import Pipeline
    return Pipeline(checkpoint_path=ckpt_dir, max_seq_len=16, target_vocab_size=300, image_size=128, n_layers=1,
                    rate=0.1, init=Init(torch.Generator().manual_seed(17)), use_graph=True)


def _batches(n):
    out = []
    g = torch.Generator().manual_seed(9)
    for _ in range(n):
        img = torch.rand(2, 128, 128, 3, generator=g) * 2 - 1
        tok = torch.randint(4, 300, (2, 16), generator=g)
        tok[:, 0] = 2
        tok[0, 9] = 3
        tok[0, 10:] = 0
        out.append((img.to(DEV), tok.to(DEV)))
    return out


def _state(pl):
    a = pl.engine.arena
    return [t.detach().clone() for t in (a.flat, a.m, a.v, a.vhat, a.step)]


def test_resume_is_bitwise_equal_to_uninterrupted(tmp_path):
    import fpnmt
    fpnmt.set_precision("bf16")
    try:
        k, m = 3, 3
        data = _batches(k + m)
        # uninterrupted k + m steps
        pa = _pipeline(None)
        la = [float(pa.train_step(*b)) for b in data]
        sa = _state(pa)
        del pa
        # k steps, checkpoint, keep going (graphs captured and live) ...
        pb = _pipeline(str(tmp_path))
        lb = [float(pb.train_step(*b)) for b in data[:k]]
        path = pb.ckpt_manager.save()
        lb_more = [float(pb.train_step(*b)) for b in data[k:]]
        assert lb + lb_more == la
        # ... then restore step k into the LIVE engine (its hipGraphs stay
        # valid: the restore copies into the arena in place) and redo m steps
        pb.ckpt.restore(path)
        lb2 = [float(pb.train_step(*b)) for b in data[k:]]
        print(f"losses uninterrupted {la}; resumed-in-place {lb2}")
        assert lb2 == la[k:]
        for x, y in zip(_state(pb), sa):
            assert torch.equal(x, y)
        del pb
        # a fresh Pipeline on the directory restores the LATEST checkpoint at
        # construction (pipeline.py:44-48): save step k again as the latest
        pc0 = _pipeline(None)
        for b in data[:k]:
            pc0.train_step(*b)
        from fpnmt.checkpoint import CheckpointManager
        CheckpointManager(pc0.ckpt, str(tmp_path / "fresh")).save()
        del pc0
        pc = _pipeline(str(tmp_path / "fresh"))
        assert int(pc.engine.arena.step) == k
        lc = [float(pc.train_step(*b)) for b in data[k:]]
        print(f"fresh-pipeline resume {lc}")
        assert lc == la[k:]
        for x, y in zip(_state(pc), sa):
            assert torch.equal(x, y)
        # train.py:96: the weights file of the resumed model reloads exactly
        wpath = str(tmp_path / "w.safetensors")
        pc.transformer.save_weights(wpath)
        pd = _pipeline(None)
        pd.transformer.load_weights(wpath)
        for (n1, p1), (n2, p2) in zip(pc.transformer.state_dict().items(), pd.transformer.state_dict().items()):
            assert n1 == n2 and torch.equal(p1, p2), n1
        assert all(math.isfinite(x) for x in la)
    finally:
        fpnmt.set_precision("fp32")
