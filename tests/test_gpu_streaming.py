"""Streaming causal inference (conv-tasnet_amd/streaming.py, csrc/ctn_stream.hip):
chunk by chunk, with per-block ring state, against (1) the REFERENCE's causal model
output (tests/golden/model_causal_cln.npz: jwr1995/Conv-TasNet's ConvTasNet, paper
dims, causal cLN, L=16, captured by make_golden.py) and (2) the whole-signal forward
of the same model on the HIP path (conv_tasnet.py:45-60 with causal=True).  fp32:
every streamed op is per frame or looks backward only, so the match is to rounding
(1e-4 relative L2 against the reference, 1e-5 against the HIP fp32 forward).  GPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import ctn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _model(norm="cLN", mask="relu", C=2, L=16, seed=0):
    import conv_tasnet as ct
    torch.manual_seed(seed)
    m = ct.ConvTasNet(N=32, L=L, B=16, H=32, P=3, X=4, R=2, C=C, norm_type=norm, causal=True,
                      mask_nonlinear=mask).to(DEV)
    with torch.no_grad():   # non-trivial norm affines
        for n, p in m.named_parameters():
            if n.endswith("gamma") or n.endswith("beta") or n.endswith(".weight") and p.dim() == 1:
                p.add_(0.2 * torch.randn_like(p))
    return m.eval()


@pytest.mark.parametrize("chunk", [16, 333, 1000, 8000])
def test_stream_matches_reference_causal_model(chunk):
    """The reference's own causal cLN model (paper dims, L=16) streamed in chunks: the
    concatenated output equals the reference's whole-signal output."""
    import conv_tasnet as ct
    import streaming
    g = np.load(os.path.join(GOLDEN, "model_causal_cln.npz"))
    N, L_, B, H, P, X, R, C = [int(v) for v in g["cfg"]]
    cfg = O.Cfg(N, L_, B, H, P, X, R, C, str(g["cfg_norm"]), bool(int(g["cfg_causal"])), str(g["cfg_mask"]))
    m = ct.ConvTasNet(N, L_, B, H, P, X, R, C, norm_type=cfg.norm_type, causal=cfg.causal,
                      mask_nonlinear=cfg.mask_nonlinear)
    m.load_state_dict(O.init_params(cfg, int(g["seed"])), strict=False)
    m = m.to(DEV).eval()
    mix = torch.from_numpy(g["mix"]).to(DEV)
    out = streaming.StreamingSeparator(m).separate(mix, chunk)
    ref = torch.from_numpy(g["est"]).to(DEV)
    assert out.shape == ref.shape
    for c in range(C):
        assert rel(out[:, c], ref[:, c]) < 1e-4, (chunk, c, rel(out[:, c], ref[:, c]))


@pytest.mark.parametrize("chunk", [8, 100, 1000, 777, 4000])
def test_stream_matches_full_forward_fp32(chunk):
    import streaming
    m = _model()
    mix = torch.randn(3, 4000, device=DEV)
    with torch.no_grad():
        full = m(mix)
    out = streaming.StreamingSeparator(m).separate(mix, chunk)
    assert out.shape == full.shape
    for c in range(full.shape[1]):
        assert rel(out[:, c], full[:, c]) < 1e-5, (chunk, c)


def test_stream_ragged_chunks_softmax_3spk_small_calls():
    """Ragged chunk sizes (1 sample to 1500), softmax mask, 3 speakers, and calls cut to
    at most 5 frames so that ring slots wrap many times."""
    import streaming
    m = _model(mask="softmax", C=3, L=20)
    mix = torch.randn(2, 3210, device=DEV)
    with torch.no_grad():
        full = m(mix)
    s = streaming.StreamingSeparator(m, max_frames=5)
    sizes, parts, i = [1, 9, 10, 333, 2, 1500, 64], [], 0
    k = 0
    while i < mix.shape[1]:
        n = sizes[k % len(sizes)]
        parts.append(s.push(mix[:, i:i + n]))
        i, k = i + n, k + 1
    parts.append(s.flush())
    out = torch.cat(parts, dim=2)
    n = out.shape[2]
    assert n == (((3210 - 20) // 10 + 1) - 1) * 10 + 20        # (K-1)*L/2 + L samples
    assert rel(out, full[:, :, :n]) < 1e-5
    assert float(full[:, :, n:].abs().max()) == 0.0 if n < 3210 else True


def test_stream_batchnorm_eval():
    import streaming
    m = _model(norm="BN")
    with torch.no_grad():   # running statistics away from (0, 1)
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.normal_(0, 0.3)
                mod.running_var.uniform_(0.5, 2.0)
    mix = torch.randn(2, 2400, device=DEV)
    with torch.no_grad():
        full = m(mix)
    out = streaming.StreamingSeparator(m).separate(mix, 250)
    assert rel(out, full) < 1e-5


def test_stream_rejects_non_streamable_models():
    import conv_tasnet as ct
    import streaming
    with pytest.raises(ValueError):
        streaming.StreamingSeparator(ct.ConvTasNet(16, 16, 8, 16, 3, 2, 1, 2, norm_type="cLN", causal=False).to(DEV))
    with pytest.raises(ValueError):
        streaming.StreamingSeparator(ct.ConvTasNet(16, 16, 8, 16, 3, 2, 1, 2, norm_type="gLN", causal=True).to(DEV))
    m = ct.ConvTasNet(16, 16, 8, 16, 3, 2, 1, 2, norm_type="BN", causal=True).to(DEV)
    with pytest.raises(ValueError):
        streaming.StreamingSeparator(m.train())


def test_stream_push_after_flush_starts_a_new_stream():
    """flush() leaves the streamer reset: pushing the same signal again reproduces the
    first stream exactly (no stale rings, tail or pending samples)."""
    import streaming
    m = _model()
    mix = torch.randn(2, 2000, device=DEV)
    s = streaming.StreamingSeparator(m)
    first = torch.cat([s.push(mix[:, :700]), s.push(mix[:, 700:]), s.flush()], dim=2)
    second = torch.cat([s.push(mix[:, :700]), s.push(mix[:, 700:]), s.flush()], dim=2)
    assert torch.equal(first, second)
    with pytest.raises(ValueError):
        streaming.StreamingSeparator(m, act_dtype=torch.bfloat16)


@pytest.mark.parametrize("norm,mask,C", [("cLN", "relu", 2), ("BN", "softmax", 3)])
def test_stream_one_call_matches_stage_entries(norm, mask, C):
    """ctn_stream_call (ABI v7: the whole call in one entry, 1x1 convs split over 32-output
    column chunks, per-frame norms recomputed by every chunk) against the v5 per-stage
    entries on the same chunks: the same arithmetic with the 1x1 sums added in another
    order, so the outputs agree to fp32 rounding, and the carried state stays in step."""
    import streaming
    m = _model(norm=norm, mask=mask, C=C)
    if norm == "BN":
        m.eval()
    mix = torch.randn(2, 3000, device=DEV)
    outs = []
    for one in (True, False):
        s = streaming.StreamingSeparator(m, max_frames=7)
        s.one_call = one
        parts = [s.push(mix[:, i:i + 333]) for i in range(0, 3000, 333)]
        parts.append(s.flush())
        outs.append(torch.cat(parts, dim=2))
    assert outs[0].shape == outs[1].shape
    assert rel(outs[0], outs[1]) < 1e-5, rel(outs[0], outs[1])


def test_stream_graph_replay_matches_direct_launches(monkeypatch):
    """ctn_stream_call replays a captured graph per argument set, reading the call's first
    frame index from the workspace (CTN_STREAM_GRAPH=1, the default); with direct
    launches (=0) every output bit is the same, over calls that reuse graphs (equal
    chunks, both tail buffers), a ragged last chunk (another K: another graph) and a
    second stream after flush()."""
    import streaming
    m = _model()
    mix = torch.randn(3, 4000, device=DEV)
    outs = []
    for g in ("1", "0"):
        monkeypatch.setenv("CTN_STREAM_GRAPH", g)
        s = streaming.StreamingSeparator(m, max_frames=8)
        parts = []
        for rep in range(2):
            parts += [s.push(mix[:, i:i + 320]) for i in range(0, 4000, 320)]
            parts.append(s.flush())
        outs.append(torch.cat(parts, dim=2))
    assert torch.equal(outs[0], outs[1])


def test_stream_refresh_weights_mid_stream():
    """refresh_weights() in the middle of a stream (the one-call path cached its
    model struct by the rings only and then replayed a graph over freed weight copies):
    after the refresh the one-call streamer must equal the per-stage entries (which rebuild
    their pointers on every call) running the same pushes and the same refresh."""
    import streaming
    mix = torch.randn(2, 3000, device=DEV)
    outs = []
    for one in (True, False):
        m = _model(seed=5)
        s = streaming.StreamingSeparator(m, max_frames=8)
        s.one_call = one
        parts = [s.push(mix[:, i:i + 320]) for i in range(0, 1600, 320)]
        with torch.no_grad():
            for p in m.parameters():
                p.mul_(0.9)
        s.refresh_weights()
        torch.cuda.empty_cache()   # the old snapshot's memory goes back to the device pool
        junk = [torch.randn(1 << 20, device=DEV) for _ in range(4)]   # and gets reused
        parts += [s.push(mix[:, i:i + 320]) for i in range(1600, 3000, 320)]
        parts.append(s.flush())
        del junk
        outs.append(torch.cat(parts, dim=2))
    assert rel(outs[0], outs[1]) < 1e-5, rel(outs[0], outs[1])


def test_stream_staging_is_bounded():
    """Pushes of many different lengths keep at most 8 staging buffer sets (the library's
    graph cache holds 8 argument sets)."""
    import streaming
    m = _model()
    s = streaming.StreamingSeparator(m, max_frames=64)
    mix = torch.randn(1, 20000, device=DEV)
    i = 0
    for n in range(40, 800, 40):
        s.push(mix[:, i:i + n])
        i += n
    assert len(s._stage) <= 8
