"""Host-side logic of the grouped projections (no GPU): DenseGroup
membership and the arena order that makes each group's kernels / biases one
contiguous block."""
import math

import torch


def _model(num_layers=2):
    from fpnmt.layers import Init
    from models.transformer import Transformer
    torch.manual_seed(0)
    return Transformer(num_layers, 512, 8, 2048, math.ceil(128 / 16) ** 2, 100, 0.0, max_seq_len=8,
                       init=Init(torch.Generator().manual_seed(0)))


def test_group_membership():
    from common.common_definitions import NUM_OF_PYRAMIDS
    m = _model(2)
    enc, dec = m.encoder, m.decoder
    assert len(enc.kv_groups) == NUM_OF_PYRAMIDS - 1
    g = enc.kv_groups[1]
    assert g.layers == [enc.enc_layers[0].mhas[1].wk, enc.enc_layers[0].mhas[1].wv,
                        enc.enc_layers[1].mhas[1].wk, enc.enc_layers[1].mhas[1].wv]
    assert enc.enc_layers[0].q_group.layers == [mh.wq for mh in enc.enc_layers[0].mhas]
    assert dec.dec_layers[1].qkv_group.layers == [dec.dec_layers[1].mha1.wq, dec.dec_layers[1].mha1.wk,
                                                  dec.dec_layers[1].mha1.wv]
    assert dec.cross_kv_group.n == 4
    # every Dense belongs to at most one group
    seen = set()
    for mod in m.modules():
        grp = mod.__dict__.get("_group")
        if grp is not None:
            assert id(mod) not in seen
            seen.add(id(mod))


def test_arena_order_contiguous():
    from fpnmt.arena import ParamArena
    from fpnmt.layers import group_param_order
    m = _model(2)
    named = [(n, p) for n, p in m.named_parameters() if p.requires_grad]
    order = group_param_order(m, named)
    assert sorted(n for n, _ in order) == sorted(n for n, _ in named)
    arena = ParamArena(order, "cpu", sparse_names=["decoder.embedding.embeddings"])
    groups = list(m.encoder.kv_groups) + [m.decoder.cross_kv_group] + \
        [l.q_group for l in m.encoder.enc_layers] + [l.qkv_group for l in m.decoder.dec_layers]
    for g in groups:
        kg, bg = g.grad_views()
        assert kg is not None and bg is not None
        for i, layer in enumerate(g.layers):
            assert kg[i].data_ptr() == layer.kernel.grad.data_ptr()
            assert bg[i * g.fout:].data_ptr() == layer.bias.grad.data_ptr()
        assert g.bias_cat().data_ptr() == g.layers[0].bias.data_ptr()
        assert torch.equal(g.bias_cat(), torch.cat([l.bias.detach() for l in g.layers]))
    # parameters keep their values through the arena adoption
    ref = _model(2)
    for (n, p), (n2, p2) in zip(m.named_parameters(), ref.named_parameters()):
        assert n == n2 and torch.equal(p.detach(), p2.detach())


def test_unordered_params_fall_back():
    m = _model(1)
    g = m.decoder.cross_kv_group
    for layer in g.layers:
        layer.kernel.grad = torch.zeros_like(layer.kernel)
        layer.bias.grad = torch.zeros_like(layer.bias)
    kg, bg = g.grad_views()
    assert kg is None and bg is None  # separate allocations: per-member fallback
    assert torch.equal(g.bias_cat(), torch.cat([l.bias.detach() for l in g.layers]))


def test_new_group_dtype_marks_members_stale():
    """A compute dtype first used after training (e.g. the fp32 parity check
    after bf16 graph steps) allocates a fresh stacked operand for the whole
    group: every member must be re-prepared, not only the first one asked."""
    from fpnmt import layers as fl
    m = _model(1)
    g = m.decoder.dec_layers[0].qkv_group
    for lay in g.layers:
        lay._gen = fl._GEN[0]  # "up to date" for the dtypes it already has
    g.ensure(torch.float64)
    assert all(lay._gen == -1 for lay in g.layers)
    assert all(torch.float64 in lay._copies for lay in g.layers)
