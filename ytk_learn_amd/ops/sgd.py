"""Column-ordered mini-batch SGD steps for the linear / FM / FFM models (GPU).

The optimizer's batches are fixed row ranges of the rank's CSR shard (only their visiting
order is shuffled per epoch), so each batch's column order is built ONCE at set-up: a
:class:`~ytk_learn_amd.ops.sparse.SparseMatrix` of the batch rows (global feature ids, one
untiled CSC over the batch) plus the list of the features the batch touches with their chunk
ranges and entry counts. A step is then

  1. the row pass (``fm_forward``; FFM: + the pair forward) on the batch rows, read in place;
  2. c_r = weight_r * l'(z_r) (fused row-loss pass, no host read);
  3. the column pass over the batch CSC chunks (``fm_backward_kernel``: sum c x S, sum c x,
     sum c x^2 per chunk; FFM: + the streamed pair-gradient kernel);
  4. ``sgd_apply_kernel``: every touched feature sums its chunks in order and updates its
     weights once -- w, V (FM / FFM, with l2 decay) and the bf16 / transposed working copies.

FFM with fixed-layout rows and k == 4 (Criteo shape) takes the pair-term path instead of
steps 3-4: the pair forward also writes E[entry][q] = x_p x_q V[i_q, f_p] for every ordered
pair of the row (both factors are in registers for the dot product), and one column kernel
(``ffm_sgd_ecol_kernel``) sums c_row * E rows per chunk -- full-line reads instead of the 16-B
V gathers of ``ffm_sgd_grad_kernel`` -- and applies the step of every column with a single
chunk in place; ``sgd_apply`` then runs over the multi-chunk columns only. E costs
entries x m x 16 B (1.7 GB for a 65536-row, 40-field batch; ``YTK_SGD_FFM_E_GB`` caps it).

Against the per-entry Hogwild! float atomics this replaces (42M atomics per 65536-row FM
batch, 409M for FFM: ``docs/performance.md``), no two threads ever write one weight, the
step is deterministic, and the per-feature mean step (``optimization.sgd.average =
feature``) takes its counts from the CSC column lengths instead of a count + clear pass.
Semantics: a synchronous mini-batch step -- every row's gradient is taken at the weights the
batch started from (the CPU reference ``fm_sgd_update`` / :func:`ffm_step_cpu` does the same).
Per-sample math: ``FMHoagOptimizer.java:127-137``, ``FFMHoagOptimizer.java:149-187``.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from ._ext import check_cuda, hip, ptr, stream
from .sparse import SparseMatrix


FFM_VT = os.environ.get("YTK_SGD_FFM_VT", "0") == "1"
# fixed-layout FFM with k == 4: the forward writes the pair terms E (entries x m x 16 B) and
# the chunk sums read them back (ffm_sgd_ecol) -- unless E would exceed this many GB
FFM_E_GB = float(os.environ.get("YTK_SGD_FFM_E_GB", 16))
SGD_CHUNK = 64  # entries per batch CSC chunk: a batch's hot columns (the bias: every row) are
#                split so no chunk's serial walk outlasts the rest of the column pass


class SGDBatch:
    """One batch's column structure (device tensors)."""

    __slots__ = ("b", "e", "o0", "X", "ucol", "ucp", "ucnt", "nu", "fields", "lay", "chunk_fa", "chunk_col",
                 "perm", "solo", "multi")


def build_batches(X: SparseMatrix, bounds, fields: Optional[torch.Tensor] = None, nfield: int = 0,
                  skip_feat: int = -1) -> List[SGDBatch]:
    """Set-up of every batch [b, e) of ``bounds`` (rows of ``X``)."""
    from .ffm import _csc_layout, _fixed_layout
    out = []
    for b, e in bounds:
        o0, o1 = int(X.indptr[b]), int(X.indptr[e])
        ip = (X.indptr[b:e + 1] - o0).contiguous()
        Xb = SparseMatrix(ip, X.indices[o0:o1], X.values[o0:o1], X.ncols, row_tile=False, chunk=SGD_CHUNK)
        counts = Xb.colptr[1:] - Xb.colptr[:-1]
        u = torch.nonzero(counts).flatten()
        bt = SGDBatch()
        bt.b, bt.e, bt.o0, bt.X = b, e, o0, Xb
        bt.perm = bt.solo = bt.multi = None
        bt.ucol = u.to(torch.int32).contiguous()
        bt.ucnt = counts[u].to(torch.int32).contiguous()
        # chunks of consecutive touched features are contiguous (empty columns own none)
        bt.ucp = torch.cat([Xb.chunk_ptr[u], Xb.chunk_ptr[-1:]]).contiguous()
        bt.nu = int(u.numel())
        bt.fields = bt.lay = bt.chunk_fa = bt.chunk_col = None
        if fields is not None:
            bt.fields = fields[o0:o1].contiguous()
            fl = _fixed_layout(Xb, bt.fields, nfield) if Xb.n > 0 else None
            if fl is not None and fl[1] <= 64:
                # fixed-layout rows: ffm_sgd_grad_kernel (field of each chunk's column; the
                # skipped feature's chunks marked -1)
                bt.lay = fl
                fa = bt.fields[Xb.csc_perm[Xb.chunk_beg]].to(torch.int32)
                col = Xb.chunk_col.to(torch.int32)
                if skip_feat >= 0:
                    fa = torch.where(col == skip_feat, torch.full_like(fa, -1), fa)
                bt.chunk_fa, bt.chunk_col = fa.contiguous(), col.contiguous()
                bt.perm = Xb.csc_perm.to(torch.int32).contiguous()  # CSC entry -> batch CSR position
                Xb.csc_perm = None
            else:
                _csc_layout(Xb, bt.fields, nfield)  # packed codes of the general pair-gradient kernel
        else:
            Xb.csc_perm = None  # only the general FFM kernel reads the entries' CSR positions
        Xb.chunk_col = None
        Xb.rows_of_nnz = None   # set-up only
        out.append(bt)
    return out


def apply_step(bt: SGDBatch, part: torch.Tensor, lat: Optional[torch.Tensor], J: int, w_lin: torch.Tensor,
               V: Optional[torch.Tensor], k: int, lr: float, l2w: float, l2v: float, reg_skip: int, upd_w: bool,
               bias_latent: bool, avg: bool, Vb: Optional[torch.Tensor] = None, Vt: Optional[torch.Tensor] = None,
               multi: bool = False):
    """``sgd_apply_kernel`` over the batch's touched features (see csrc/hip/fm.hip); ``multi``:
    only the columns of more than one chunk (the pair-term path updated the others)."""
    check_cuda(part, w_lin, *(t for t in (lat, V, Vb, Vt) if t is not None))
    if multi:
        ucol, ucb, uce, ucnt, nu = bt.multi
        if nu == 0:
            return
    else:
        ucol, ucb, uce, ucnt, nu = bt.ucol, bt.ucp, bt.ucp[1:], bt.ucnt, bt.nu
    hip().sgd_apply(ptr(ucol), ptr(ucb), ptr(uce), ptr(ucnt), nu, ptr(part), int(part.shape[1]),
                    ptr(lat) if lat is not None else 0, int(J), ptr(w_lin), ptr(V) if V is not None else 0, int(k),
                    ptr(Vb) if Vb is not None else 0, ptr(Vt) if Vt is not None else 0, int(w_lin.numel()),
                    float(lr), float(l2w), float(l2v), int(reg_skip), 1 if upd_w else 0, 1 if bias_latent else 0,
                    1 if avg else 0, stream(w_lin))


def column_sums(bt: SGDBatch, c: torch.Tensor, S: Optional[torch.Tensor], k: int) -> torch.Tensor:
    """part[chunk, k + 2] = [sum c x S_f | sum c x | sum c x^2] over the batch CSC chunks."""
    Xb = bt.X
    part = torch.empty((max(Xb.n_chunks, 1), k + 2), dtype=torch.float32, device=c.device)
    hip().fm_backward(ptr(Xb.chunk_bounds), ptr(Xb.chunk_end_b), Xb.n_chunks, ptr(Xb.csc_rows), ptr(Xb.csc_vals),
                      ptr(c), ptr(S) if (S is not None and k > 0) else 0, k, ptr(part), stream(c))
    return part


def ffm_pair_sums(bt: SGDBatch, c: torch.Tensor, V: torch.Tensor, Vt: Optional[torch.Tensor], nfield: int, k: int,
                  skip_feat: int) -> torch.Tensor:
    """lat[chunk, nfield * k] = the chunk's FFM pair gradient: ffm_sgd_grad_kernel over the
    model's V ([F][nfield][k]) for fixed-layout batches, else the general column-ordered kernel
    over the transposed copy Vt ([nfield][F][k])."""
    from .ffm import _csc_layout
    Xb = bt.X
    J = nfield * k
    lat = torch.empty((max(Xb.n_chunks, 1), J), dtype=torch.float32, device=c.device)
    h, s = hip(), stream(c)
    if bt.lay is not None and k in (4, 8):
        lay_field, m = bt.lay
        # YTK_SGD_FFM_VT=1 (with the field-major copy allocated): gather from Vt instead of V
        src, vt_nfeat = (Vt, Xb.ncols) if (Vt is not None and FFM_VT) else (V, 0)
        h.ffm_sgd_grad(ptr(Xb.chunk_bounds), ptr(Xb.chunk_end_b), Xb.n_chunks, ptr(Xb.csc_rows), ptr(Xb.csc_vals),
                       ptr(bt.chunk_fa), ptr(bt.chunk_col), ptr(Xb.indices), 0 if Xb.one_hot else ptr(Xb.values), m,
                       ptr(lay_field), ptr(c), ptr(src), nfield, k, ptr(lat), vt_nfeat, int(skip_feat), s)
        return lat
    if Vt is None:
        raise RuntimeError("ffm sgd: the general pair-gradient kernel needs the transposed latents")
    lay = _csc_layout(Xb, bt.fields, nfield)
    if lay is None:
        raise RuntimeError("ffm sgd: feature / field codes do not fit 32 bits")
    distinct, code, sh, vals = lay
    h.ffm_grad_csc(ptr(Xb.chunk_bounds), ptr(Xb.chunk_end_b), Xb.n_chunks, ptr(Xb.csc_rows), ptr(Xb.csc_vals),
                   ptr(Xb.csc_perm), ptr(Xb.indptr), ptr(code), sh, ptr(vals) if vals is not None else 0,
                   ptr(Vt), Xb.ncols, nfield, k, ptr(c), ptr(lat), int(skip_feat), int(distinct), s)
    return lat


def pair_terms_elems(batches: List[SGDBatch], V: torch.Tensor, k: int, elem_bytes: int = 4) -> int:
    """Elements of the pair-term buffer E when every batch takes the E path (fixed layout, k ==
    4, V 16-B aligned, E within YTK_SGD_FFM_E_GB at ``elem_bytes`` per element), else 0."""
    if FFM_E_GB <= 0 or FFM_VT or k != 4 or V.data_ptr() % 16 or not batches:
        return 0
    if any(bt.lay is None for bt in batches):
        return 0
    m = batches[0].lay[1]
    n = max(bt.X.nnz for bt in batches) * m * 4
    return n if n * elem_bytes <= FFM_E_GB * (1 << 30) else 0


def ffm_forward_e(bt: SGDBatch, indptr, idx, val, fld, V: torch.Tensor, nfield: int, skip_feat: int,
                  E: torch.Tensor, Vb: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Pair sums of the batch rows (float32 [n]) + their pair terms into E (ffm_pairs_k4_kernel<true>).
    ``Vb`` (bf16 working copy of V; E is then bf16): the LDS-staged kernel reads it instead of V."""
    from .ffm import lds_forward_ok
    n = bt.e - bt.b
    out = torch.empty(n, dtype=torch.float32, device=V.device)
    check_cuda(indptr, idx, val, fld, V, E)
    m = int(bt.lay[1])
    if Vb is not None:
        if not (lds_forward_ok(m, nfield, 4, V) and E.dtype == torch.bfloat16):
            raise RuntimeError("ffm sgd bf16: needs the LDS-staged pair forward (k = 4, rows of <= 64 entries)")
        hip().ffm_pairs_lds(ptr(indptr), ptr(idx), ptr(val), ptr(fld), n, ptr(Vb), nfield, ptr(out), int(skip_feat),
                            m, ptr(E), int(bt.o0), 1, stream(V))
        return out
    if lds_forward_ok(m, nfield, 4, V):  # the row's latent rows staged in LDS (ffm_pairs_lds_kernel<true>)
        hip().ffm_pairs_lds(ptr(indptr), ptr(idx), ptr(val), ptr(fld), n, ptr(V), nfield, ptr(out), int(skip_feat), m,
                            ptr(E), int(bt.o0), 0, stream(V))
        return out
    hip().ffm_pairs_fwd_e(ptr(indptr), ptr(idx), ptr(val), ptr(fld), n, ptr(V), nfield, ptr(out), int(skip_feat),
                          ptr(E), int(bt.o0), int(bt.lay[1]), stream(V))
    return out


def prepare_pair_terms(bt: SGDBatch):
    """Set-up of the pair-term path: solo[chunk] = its column has no other chunk (updated by
    ffm_sgd_ecol_kernel itself), and the multi-chunk columns (ucol, chunk begin, chunk end,
    count, n) left to sgd_apply."""
    nch_u = bt.ucp[1:] - bt.ucp[:-1]  # chunks per touched column (contiguous, in column order)
    bt.solo = (torch.repeat_interleave(nch_u, nch_u) == 1).to(torch.uint8).contiguous()
    mu = nch_u > 1
    bt.multi = (bt.ucol[mu].contiguous(), bt.ucp[:-1][mu].contiguous(), bt.ucp[1:][mu].contiguous(),
                bt.ucnt[mu].contiguous(), int(mu.sum()))


def ffm_step_e(bt: SGDBatch, c: torch.Tensor, E: torch.Tensor, w_lin: torch.Tensor, V: torch.Tensor, nfield: int,
               k: int, lr: float, l2w: float, l2v: float, reg_skip: int, upd_w: bool, bias_latent: bool, avg: bool,
               Vb: Optional[torch.Tensor] = None):
    """ffm_sgd_ecol_kernel: the step of every single-chunk column; returns (lin, lat), the
    multi-chunk columns' chunk partials for :func:`apply_step` (``multi=True``). ``Vb``: E is
    bf16 and the bf16 working copy of every updated latent slot is re-rounded."""
    Xb = bt.X
    lay_field, m = bt.lay
    nch = max(Xb.n_chunks, 1)
    lat = torch.empty((nch, nfield * k), dtype=torch.float32, device=c.device)
    lin = torch.empty((nch, 2), dtype=torch.float32, device=c.device)
    check_cuda(c, E, w_lin, V)
    hip().ffm_sgd_ecol(ptr(Xb.chunk_bounds), ptr(Xb.chunk_end_b), Xb.n_chunks, ptr(Xb.csc_rows), ptr(Xb.csc_vals),
                       ptr(bt.perm), ptr(bt.chunk_fa), ptr(bt.chunk_col), ptr(bt.solo), ptr(E), m, ptr(lay_field),
                       ptr(c), ptr(lat), ptr(lin), ptr(w_lin), ptr(V), float(lr), float(l2w), float(l2v),
                       int(reg_skip), 1 if upd_w else 0, 1 if bias_latent else 0, 1 if avg else 0,
                       ptr(Vb) if Vb is not None else 0, stream(c))
    return lin, lat


def needs_transposed(batches: List[SGDBatch], V: torch.Tensor, k: int) -> bool:
    """Whether some batch takes the general pair-gradient kernel (which reads Vt)."""
    return FFM_VT or any(bt.lay is None for bt in batches) or k not in (4, 8)


def _ffm_pair_grad_bf16(indptr, idx, x, fld, Vb: torch.Tensor, nfield: int, k: int, c, gV, skip_feat: int):
    """gV[i_p, f_q] += c_r bf16(x_p x_q Vb[i_q, f_p]) over the ordered pairs p != q of every row --
    the GPU bf16 path's pair terms (ffm_pairs_lds_kernel<true, true>) rounded where it rounds."""
    n = int(indptr.shape[0] - 1)
    lens = (indptr[1:] - indptr[:-1]).long()
    rows = torch.repeat_interleave(torch.arange(n), lens)
    nnz = rows.numel()
    ent = torch.arange(nnz)
    cnts = lens[rows]
    e1 = torch.repeat_interleave(ent, cnts)
    first = torch.cumsum(cnts, 0) - cnts
    e2 = (indptr[rows].long() - indptr[0].long())[e1] + (torch.arange(e1.numel()) - torch.repeat_interleave(first, cnts))
    ii, ff = idx.long(), fld.long()
    keep = (e1 != e2) & (ii[e1] != skip_feat) & (ii[e2] != skip_feat)
    e1, e2 = e1[keep], e2[keep]
    V3 = Vb.float().view(-1, nfield, k)
    t = ((x[e1] * x[e2])[:, None] * V3[ii[e2], ff[e1]]).to(torch.bfloat16).float()
    G3 = gV.view(-1, nfield, k)
    G3.index_put_((ii[e1], ff[e2]), c[rows[e1]][:, None] * t, accumulate=True)


def ffm_step_cpu(indptr, idx, val, fld, w_lin, V, nfield: int, k: int, c, lr: float, l2w: float, l2v: float,
                 reg_skip: int, upd_w: bool, bias_latent: bool, cnt=None, skip_feat: int = -1, Vb=None):
    """CPU reference of one synchronous FFM batch step (linear part + pairs + l2 decay), all
    gradients at the batch's starting weights; ``cnt`` (int32 [F]): per-feature mean; ``Vb``
    (bf16 copy of V): the pair terms come from it, rounded to bf16 (the GPU bf16 path)."""
    from .ffm import ffm_backward
    n = int(indptr.shape[0] - 1)
    b0, e0 = int(indptr[0]), int(indptr[-1])
    rows = torch.repeat_interleave(torch.arange(n), (indptr[1:] - indptr[:-1]).long())
    ix = idx[b0:e0].long()
    x = val[b0:e0]
    F = w_lin.numel()
    ones = torch.ones_like(x)
    ent = torch.zeros(F).index_add_(0, ix, ones)  # entries per feature in the batch
    div = cnt.clamp(min=1).float() if cnt is not None else torch.ones(F)
    gw = torch.zeros(F).index_add_(0, ix, c[rows] * x)
    is_bias = torch.zeros(F, dtype=torch.bool)
    if reg_skip >= 0:
        is_bias[reg_skip] = True
    gw += torch.where(is_bias, torch.zeros(()), ent * l2w * w_lin)
    if not upd_w:
        gw = torch.where(is_bias, gw, torch.zeros(()))
    if V is not None and nfield * k > 0:
        gV = torch.zeros_like(V)
        ip_rel = indptr - b0
        if Vb is not None:
            _ffm_pair_grad_bf16(ip_rel, idx[b0:e0], x, fld[b0:e0], Vb, nfield, k, c, gV, skip_feat)
        else:
            ffm_backward(ip_rel, idx[b0:e0], x, fld[b0:e0], V, nfield, k, c, gV, skip_feat=skip_feat)
        G2 = gV.view(F, -1)
        V2 = V.view(F, -1)
        G2 += torch.where(is_bias[:, None], torch.zeros(()), (ent * l2v)[:, None] * V2)
        if not bias_latent and reg_skip >= 0:
            G2[reg_skip] = 0.0
        V2 -= (lr / div)[:, None] * G2 * (ent > 0)[:, None]
    w_lin -= (lr / div) * gw
