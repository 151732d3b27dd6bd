"""Column-ordered synchronous mini-batch SGD (ops/sgd.py, sgd_apply_kernel).

CPU: the synchronous step equals its definition (every gradient at the batch's starting
weights) written out per sample, for linear / FM / FFM with l2 decay, the bias rule and both
averaging modes. GPU: the four-kernel step (row pass, row loss, column pass + pair gradient,
sgd_apply) equals the CPU reference step on the same data, batch after batch.
"""
import numpy as np
import pytest
import torch

from ytk_learn_amd.config.params import CommonParams
from ytk_learn_amd.data.dataflow import SparseData
from ytk_learn_amd.data.synthetic import criteo_like
from ytk_learn_amd.models.continuous.base import LoadedData
from ytk_learn_amd.optim.sgd import SGDOptimizer, SGDParams
from ytk_learn_amd.utils.logging import YtkLogger


def _model(name, n=3000, nf=6, feats=240, k=4, dev="cpu", seed=5, uneven=False, pad=0):
    ip, ix, vv, fl, y = criteo_like(n, nf, feats, seed=seed)
    g = torch.Generator().manual_seed(seed)
    vv = (0.5 + torch.rand(vv.shape, generator=g)).contiguous()
    F = nf * (feats // nf) + 1 + pad  # pad: unused features (F % 4 == 0 puts V 16-B aligned)
    # bias column 0 in front of every row (as the data loader lays it out)
    m = nf
    ip2 = torch.arange(n + 1, dtype=torch.int64) * (m + 1)
    idx2 = torch.zeros(n * (m + 1), dtype=torch.int32)
    val2 = torch.ones(n * (m + 1), dtype=torch.float32)
    fld2 = torch.zeros(n * (m + 1), dtype=torch.int32)
    sel = torch.ones(n * (m + 1), dtype=torch.bool)
    sel[::m + 1] = False
    idx2[sel] = ix + 1
    val2[sel] = vv
    fld2[sel] = fl + 1
    if uneven:  # drop some entries: rows of different lengths, not every field present
        keep = torch.rand(idx2.shape, generator=g) > 0.2
        keep[::m + 1] = True
        rows = torch.repeat_interleave(torch.arange(n), m + 1)
        idx2, val2, fld2 = idx2[keep], val2[keep], fld2[keep]
        cnt = torch.zeros(n, dtype=torch.int64).index_add_(0, rows[keep], torch.ones(int(keep.sum()), dtype=torch.int64))
        ip2 = torch.zeros(n + 1, dtype=torch.int64)
        ip2[1:] = torch.cumsum(cnt, 0)
    w = torch.ones(n)
    d = SparseData(ip2.to(dev), idx2.to(dev), val2.to(dev), y.to(dev), w.to(dev),
                   fld2.to(dev) if name == "ffm" else None, None, float(n), float(n), float(n))
    p = CommonParams()
    p.loss.loss_function = "sigmoid"
    p.loss.evaluate_metric = []
    p.model.need_bias = True
    p.model.data_path = "/tmp/ytk_test_sgd_column"
    p.extra = {"k": [1, k], "bias_need_latent_factor": False}
    names = ["_bias_"] + [f"f{i}" for i in range(1, F)]
    loaded = LoadedData(d, None, names, {nm: i for i, nm in enumerate(names)},
                        ["_bias_"] + [f"c{i}" for i in range(nf)])
    log = YtkLogger(0)
    log.quiet = True
    from ytk_learn_amd.parallel.comm import Comm
    comm = Comm.local(torch.device(dev))
    if name == "linear":
        from ytk_learn_amd.models.continuous.linear import LinearModel
        return LinearModel(p, loaded, comm, log)
    if name == "fm":
        from ytk_learn_amd.models.continuous.fm import FMModel
        return FMModel(p, loaded, comm, log)
    from ytk_learn_amd.models.continuous.ffm import FFMModel
    return FFMModel(p, loaded, comm, log)


def _opt(model, avg="feature", dtype="fp32", batch=512, l2=(1e-3, 2e-3)):
    log = YtkLogger(0)
    log.quiet = True
    return SGDOptimizer(model, SGDParams(learning_rate=0.2, batch_size=batch, epochs=1, average=avg, dtype=dtype),
                        [0.0, 0.0], list(l2), None, log, float(model.data.train.n), 1.0)


def _per_sample_step(model, w, b, e, lr, l2w, l2v, avg):
    """Definition: per-sample gradients at the starting weights, summed per weight, divided by
    the batch entries holding the feature (avg) -- written with explicit loops over rows."""
    F = model.F
    X = model.X
    w0 = w.clone()
    upd = torch.zeros_like(w)
    cnt = torch.zeros(F)
    ip, ix, xv = X.indptr, X.indices.long(), X.values
    fl = model.data.train.fields
    for r in range(b, e):
        s, t = int(ip[r]), int(ip[r + 1])
        ii, xx = ix[s:t], xv[s:t]
        fx = float((w0[ii] * xx).sum())
        if model.name == "fm":
            V = w0[F:].view(F, model.kk)
            S = (V[ii] * xx[:, None]).sum(0)
            fx += 0.5 * float((S * S - ((V[ii] * xx[:, None]) ** 2).sum(0)).sum())
        if model.name == "ffm":
            V = w0[F:].view(F, model.nf, model.kk)
            ff = fl[s:t].long()
            for p in range(len(ii)):
                for q in range(p + 1, len(ii)):
                    if int(ii[p]) == 0 or int(ii[q]) == 0:
                        continue
                    fx += float((V[ii[p], ff[q]] * V[ii[q], ff[p]]).sum()) * float(xx[p] * xx[q])
        y = float(model.data.train.y[r, 0])
        c = 1.0 / (1.0 + np.exp(-fx)) - y
        for p in range(len(ii)):
            i = int(ii[p])
            cnt[i] += 1
            gw = c * float(xx[p]) + (0.0 if i == 0 else l2w * float(w0[i]))
            upd[i] += gw
            if model.name == "fm" and i != 0:
                V = w0[F:].view(F, model.kk)
                gv = c * float(xx[p]) * (S - V[i] * float(xx[p])) + l2v * V[i]
                upd[F + i * model.kk:F + (i + 1) * model.kk] += gv
            if model.name == "ffm" and i != 0:
                V = w0[F:].view(F, model.nf, model.kk)
                ff = fl[s:t].long()
                gv = torch.zeros(model.nf, model.kk)
                for q in range(len(ii)):
                    if q != p and int(ii[q]) != 0:
                        gv[ff[q]] += c * float(xx[p] * xx[q]) * V[ii[q], ff[p]]
                gv += l2v * V[i]
                st = model.nf * model.kk
                upd[F + i * st:F + (i + 1) * st] += gv.reshape(-1)
    div = cnt.clamp(min=1) if avg == "feature" else torch.ones(F)
    out = w0.clone()
    out[:F] -= lr * upd[:F] / div
    J = (w.numel() - F) // F
    if J:
        out[F:] -= (lr * upd[F:].view(F, J) / div[:, None]).reshape(-1)
    return out


@pytest.mark.parametrize("name", ["linear", "fm", "ffm"])
@pytest.mark.parametrize("avg", ["feature", "none"])
def test_cpu_step_is_synchronous_per_sample_sum(name, avg):
    m = _model(name, n=40, nf=4, feats=40, k=3, uneven=True)
    opt = _opt(m, avg=avg, batch=40)
    w = m.w.clone()
    want = _per_sample_step(m, w, 0, 40, 0.2, 1e-3, 2e-3, avg)
    opt._step(w, 0, 40, 0.2)
    torch.testing.assert_close(w, want, rtol=2e-4, atol=2e-6)


def test_cpu_ffm_bf16_step_close_to_fp32():
    """The CPU emulation of the FFM bf16 path (forward from the bf16 copy, bf16 pair terms) moves
    the weights like the fp32 step up to bf16 rounding, and really rounds (not bitwise equal)."""
    outs = []
    for dt in ("fp32", "bf16"):
        m = _model("ffm", nf=9, feats=320, pad=3)
        o = _opt(m, dtype=dt)
        w = m.w.clone()
        o._sync_copy(w)
        o._step(w, 0, 512, 0.2)
        outs.append((w, m.w.clone()))
    (w32, w0), (w16, _) = outs
    d32, d16 = w32 - w0, w16 - w0
    assert not torch.equal(d32, d16)
    assert float((d16 - d32).norm() / d32.norm()) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("name,dtype,uneven,pad", [("linear", "fp32", False, 0), ("fm", "fp32", False, 0),
                                                   ("fm", "bf16", False, 0), ("ffm", "fp32", False, 0),
                                                   ("ffm", "fp32", False, 3), ("ffm", "bf16", False, 3),
                                                   ("ffm", "fp32", True, 0),
                                                   ("fm", "fp32", True, 0)])
@pytest.mark.parametrize("avg", ["feature", "none"])
def test_gpu_column_step_matches_cpu_reference(cuda, name, dtype, uneven, pad, avg):
    """Three batches through the GPU column-ordered step vs the CPU synchronous step (fp32
    sums in different orders: rtol 1e-4; bf16: the forward reads the rounded copy on both).
    FFM fixed layout: pad 0 (V unaligned) takes ffm_sgd_grad_kernel, pad 3 (F % 4 == 0) the
    forward-written pair terms + ffm_sgd_ecol_kernel; FFM bf16 (pad 3) stages the bf16 copy and
    writes bf16 pair terms -- the CPU step reads the same copy and rounds the same terms."""
    nf = 8  # the streamed FFM pair kernel needs >= 8 positions per row (ops/ffm._fixed_layout)
    if name == "ffm" and dtype == "bf16":
        nf = 9  # bf16 pair terms move slot pairs: rows of nf + 1 (bias) = 10 positions
        pad = (-(nf * (320 // nf) + 1)) % 4  # V 16-B aligned: the pair-term path (pad 3 at nf = 8)
    mc = _model(name, nf=nf, feats=320, uneven=uneven, pad=pad)
    mg = _model(name, nf=nf, feats=320, dev="cuda", uneven=uneven, pad=pad)
    oc, og = _opt(mc, avg=avg, dtype=dtype), _opt(mg, avg=avg, dtype=dtype)
    wc, wg = mc.w.clone(), mg.w.clone()
    oc._sync_copy(wc)
    og._sync_copy(wg)
    bounds = [(0, 512), (512, 1024), (2048, 2560)]
    batches = og._setup(bounds)
    if name == "ffm" and not uneven:
        assert all(bt.lay is not None for bt in batches) and og.Vt is None  # fixed-layout kernels ran
        assert (og.E is not None) == (pad == 3 or dtype == "bf16")
        if dtype == "bf16":
            assert og.Vb is not None and og.E is not None and og.E.dtype == torch.bfloat16
    for j, (b, e) in enumerate(bounds):
        oc._step(wc, b, e, 0.2)
        og._step(wg, b, e, 0.2, batches[j])
        tol = 3e-3 if dtype == "bf16" else 1e-4
        torch.testing.assert_close(wg.cpu(), wc, rtol=tol, atol=tol * 1e-2)
    if og.Vt is not None:  # the transposed working copy tracks V
        F = mg.F
        torch.testing.assert_close(og.Vt, wg[F:].view(F, mg.nf, mg.kk).transpose(0, 1), rtol=0, atol=0)
    if og.Vb is not None:
        F = mg.F
        torch.testing.assert_close(og.Vb, wg[F:].view(F, -1).to(torch.bfloat16), rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("nf,pad", [(6, 0), (8, 3)])
def test_gpu_column_step_deterministic(cuda, nf, pad):
    """No atomics: two runs of the same batches give bitwise identical weights (general pair
    kernel; fixed layout with the forward-written pair terms)."""
    outs = []
    for _ in range(2):
        m = _model("ffm", dev="cuda", nf=nf, feats=320, pad=pad)
        o = _opt(m)
        w = m.w.clone()
        o._sync_copy(w)
        bounds = [(0, 1000), (1000, 2000)]
        bts = o._setup(bounds)
        for j, (b, e) in enumerate(bounds):
            o._step(w, b, e, 0.2, bts[j])
        outs.append(w)
    assert torch.equal(outs[0], outs[1])


def _run_gpu_vs_cpu(name, nf, feats, pad, bounds, tol=1e-4, prep=None):
    mc = _model(name, nf=nf, feats=feats, pad=pad)
    mg = _model(name, nf=nf, feats=feats, dev="cuda", pad=pad)
    if prep is not None:
        prep(mc)
        prep(mg)
    oc, og = _opt(mc), _opt(mg)
    wc, wg = mc.w.clone(), mg.w.clone()
    oc._sync_copy(wc)
    og._sync_copy(wg)
    batches = og._setup(bounds)
    for j, (b, e) in enumerate(bounds):
        oc._step(wc, b, e, 0.2)
        og._step(wg, b, e, 0.2, batches[j])
        torch.testing.assert_close(wg.cpu(), wc, rtol=tol, atol=tol * 1e-2)
    return og, batches


@pytest.mark.gpu
@pytest.mark.parametrize("nf,feats", [(8, 320), (62, 620)])
def test_gpu_ffm_pair_terms_path_matches_cpu(cuda, monkeypatch, nf, feats):
    """The forward-written pair terms path (ffm_pairs_k4_kernel<true>: E through a per-wave LDS
    triangle, then ffm_sgd_ecol_kernel) against the CPU synchronous step -- taken in production
    when the LDS-staged forward does not fit (m * (nfield + 1) * 16 > 64 KiB, e.g. m near 64) or
    with YTK_FFM_LDS=0; forced here with the LDS-staged forward off, at m = 9 and m = 63."""
    import ytk_learn_amd.ops.ffm as offm
    monkeypatch.setattr(offm, "LDS_FWD", False)
    og, batches = _run_gpu_vs_cpu("ffm", nf, feats, (-(nf * (feats // nf) + 1)) % 4,
                                  [(0, 256), (256, 512)])
    assert og.E is not None and all(bt.lay is not None for bt in batches)


@pytest.mark.gpu
def test_gpu_ffm_sgd_skips_bias_pairs_with_nonzero_bias_latent(cuda):
    """bias_need_latent_factor = false excludes the bias from every pair even when its latent
    row is not zero (a model continued from one saved with a bias latent): the GPU fixed-layout
    pair gradient (ffm_sgd_grad_kernel, skip_feat) equals the CPU step, which skips it."""
    def prep(m):
        F, J = m.F, m.nf * m.kk
        m.w[F:F + J] = torch.linspace(0.5, 1.5, J, device=m.w.device)  # feature 0 = the bias

    og, batches = _run_gpu_vs_cpu("ffm", 8, 320, 0, [(0, 512), (512, 1024)], prep=prep)
    assert og.E is None and all(bt.lay is not None for bt in batches)  # ffm_sgd_grad_kernel ran
