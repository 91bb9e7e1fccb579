"""Host-side pieces of the drop-in Pipeline surface (no GPU): the Keras Mean
train-loss metric (utils/pipeline.py:35,80; train.py:47,56), the early-stop
checkpoint policy (utils/utils.py:120-154), safetensors checkpoint round trips
(utils/pipeline.py:38-48) and the CLIPNORM_MODE flag (pipeline.py:30)."""
import math

import numpy as np
import pytest
import torch


def test_mean_metric_keras_semantics():
    from utils.utils import Mean
    m = Mean(name="train_loss")
    assert float(m.result().numpy()) == 0.0  # divide_no_nan before any update
    for v in (1.0, 2.0, 6.0):
        m(torch.tensor(v))
    r = m.result()
    assert isinstance(r.numpy(), np.ndarray) and r.numpy().shape == ()
    assert float(r.numpy()) == pytest.approx(3.0)
    m.reset_states()
    assert float(m.result().numpy()) == 0.0
    m(torch.tensor([4.0, 5.0]))  # a batch of values: each weighs 1
    assert float(m.result()) == pytest.approx(4.5)


def _ref_saver_trace(accs, epochs, min_break, gap):
    """The reference rule (utils/utils.py:126-154), restated independently."""
    best, best_ep, out = -math.inf, 0, []
    for ep, acc in enumerate(accs, start=1):
        if best_ep == 0:
            best, best_ep = acc, ep
        if acc > best:
            best, best_ep = acc, ep
            out.append(1)
            continue
        if ep <= min_break:
            best, best_ep = acc, ep
            out.append(0)
            continue
        out.append(-1 if min(epochs, max(min_break, int(best_ep * 2.0)), int(best_ep + gap)) <= ep else 0)
    return out


def test_smart_checkpoint_saver_matches_reference_rule():
    from utils.utils import SmartCheckpointSaver

    class Mgr:
        saved = 0

        def save(self):
            Mgr.saved += 1
            return f"ckpt-{Mgr.saved}"

    rng = np.random.default_rng(0)
    for trial in range(20):
        accs = list(np.round(rng.random(40), 2))
        saver = SmartCheckpointSaver(Mgr(), epochs=40, min_epoch_to_break=10, gap_of_dead_epoch=5)
        got = []
        for ep, a in enumerate(accs, start=1):
            r = saver(ep, a)
            got.append(r)
            if r == -1:
                break
        want = _ref_saver_trace(accs, 40, 10, 5)[:len(got)]
        assert got == want, (trial, got, want)


def test_clipnorm_mode_flag():
    from utils.pipeline import clipnorm_for
    assert clipnorm_for("per_tensor") == 1.0
    assert clipnorm_for("none") == 0.0
    with pytest.raises(ValueError):
        clipnorm_for("global")


class _Tiny(torch.nn.Module):
    def __init__(self, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.w = torch.nn.Parameter(torch.randn(3, 5, generator=g))
        self.b = torch.nn.Parameter(torch.randn(7, generator=g))
        self.register_buffer("stat", torch.randn(4, generator=g))


class _Eng:
    def __init__(self, model):
        from fpnmt.arena import ParamArena
        self.arena = ParamArena(list(model.named_parameters()), "cpu")


def test_checkpoint_roundtrip_cpu(tmp_path):
    from fpnmt.checkpoint import Checkpoint, CheckpointManager
    m = _Tiny(0)
    eng = _Eng(m)
    a = eng.arena
    g = torch.Generator().manual_seed(5)
    for buf in (a.m, a.v, a.vhat):
        buf.copy_(torch.randn(buf.shape, generator=g))
    a.step.fill_(123)
    ck = Checkpoint(m, eng)
    mgr = CheckpointManager(ck, str(tmp_path), max_to_keep=2)
    p1 = mgr.save()
    want = {k: v.clone() for k, v in ck.state_tensors().items()}
    # a second model with other values restores to the saved state, in place
    m2 = _Tiny(1)
    eng2 = _Eng(m2)
    flat_ptr = eng2.arena.flat.data_ptr()
    mgr2 = CheckpointManager(Checkpoint(m2, eng2), str(tmp_path))
    assert mgr2.latest_checkpoint == p1
    mgr2.checkpoint.restore(mgr2.latest_checkpoint)
    got = mgr2.checkpoint.state_tensors()
    assert set(got) == set(want)
    for k in want:
        assert torch.equal(got[k], want[k]), k
    assert eng2.arena.flat.data_ptr() == flat_ptr and m2.w.data_ptr() == flat_ptr  # params still arena views
    assert int(eng2.arena.step) == 123
    # max_to_keep: the oldest file goes
    p2, p3 = mgr.save(), mgr.save()
    import os
    assert not os.path.exists(p1) and os.path.exists(p2) and os.path.exists(p3)
    assert CheckpointManager(Checkpoint(m, eng), str(tmp_path)).latest_checkpoint == p3


def test_checkpoint_rejects_mismatched_model(tmp_path):
    from fpnmt.checkpoint import Checkpoint, CheckpointManager
    m = _Tiny(0)
    p = CheckpointManager(Checkpoint(m, _Eng(m)), str(tmp_path)).save()

    class Other(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.zeros(3, 6))
            self.b = torch.nn.Parameter(torch.zeros(7))
            self.register_buffer("stat", torch.zeros(4))

    o = Other()
    with pytest.raises(ValueError):
        Checkpoint(o, _Eng(o)).restore(p)


def test_train_loop_body_drives_pipeline(monkeypatch, tmp_path):
    """train.py:46-57's per-epoch / per-batch calls (reset_states, train_step,
    result().numpy()) against the build's Pipeline with a stub dataset. The
    step itself is stubbed here (no GPU); tests/test_gpu_model.py runs it for real."""
    from fpnmt.layers import Init
    from utils.pipeline import Pipeline
    pl = Pipeline(None, str(tmp_path / "ck"), max_seq_len=8, target_vocab_size=50, image_size=64, n_layers=1,
                  device="cpu", init=Init(torch.Generator().manual_seed(0)), use_graph=False)
    losses = iter([3.0, 2.0, 1.0, 4.0])
    monkeypatch.setattr(pl.engine, "step", lambda img, tok: torch.tensor(next(losses)))
    dataset = [(torch.zeros(2, 64, 64, 3), torch.zeros(2, 8, dtype=torch.int32))] * 2
    seen = []
    for epoch in range(2):
        pl.train_loss.reset_states()
        for img, caption_token in dataset:
            pl.train_step(img, caption_token)
            seen.append(float(pl.train_loss.result().numpy()))
    assert seen == pytest.approx([3.0, 2.5, 1.0, 2.5])
    # the manager exists and saves / finds checkpoints like tf.train.CheckpointManager
    path = pl.ckpt_manager.save()
    assert pl.ckpt_manager.latest_checkpoint == path


def test_transformer_save_load_weights_cpu(tmp_path):
    """train.py:96 master.transformer.save_weights(path): every parameter and
    buffer round-trips (safetensors); load_weights restores in place."""
    import math as _m
    from fpnmt.layers import Init
    from models.transformer import Transformer
    mk = lambda seed: Transformer(1, 512, 8, 2048, _m.ceil(64 / 16) ** 2, 50, 0.0, max_seq_len=8,  # noqa: E731
                                  init=Init(torch.Generator().manual_seed(seed)))
    a, b = mk(0), mk(1)
    path = str(tmp_path / "w" / "transformer.safetensors")
    a.save_weights(path)
    ptrs = {k: v.data_ptr() for k, v in b.state_dict().items()}
    b.load_weights(path)
    sa, sb = a.state_dict(), b.state_dict()
    assert set(sa) == set(sb)
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
        assert sb[k].data_ptr() == ptrs[k], k  # in place


def test_pipeline_metric_eval_lazy(tmp_path):
    """pipeline.py:15 self.metric_eval = MetricEval(DATADIR, DATATYPE_VAL),
    used at train.py:76 as master.metric_eval(RESULT_FILE) -> CIDEr."""
    import json
    from utils.pipeline import Pipeline
    ann = tmp_path / "annotations"
    ann.mkdir()
    gt = {"images": [{"id": 1}, {"id": 2}],
          "annotations": [{"image_id": 1, "id": 1, "caption": "a dog runs on the grass"},
                          {"image_id": 1, "id": 2, "caption": "a dog is running"},
                          {"image_id": 2, "id": 3, "caption": "a cat sleeps on a sofa"},
                          {"image_id": 2, "id": 4, "caption": "the cat is sleeping"}]}
    (ann / "captions_val.json").write_text(json.dumps(gt))
    res = tmp_path / "res.json"
    res.write_text(json.dumps([{"image_id": 1, "caption": "a dog runs on the grass"},
                               {"image_id": 2, "caption": "a cat sleeps on a sofa"}]))
    pl = Pipeline.__new__(Pipeline)  # the metric needs no model
    pl._metric_eval_src, pl._metric_eval = (str(tmp_path), "val"), None
    me = pl.metric_eval
    assert me is pl.metric_eval  # built once
    cider = me(str(res))
    assert cider > 0.5 and "Bleu_4" in me.last_eval
