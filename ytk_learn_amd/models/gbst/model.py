"""Gradient-boosted soft trees: gbmlr, gbsdt, gbhmlr, gbhsdt.

Each "tree" is a K-expert mixture fitted by L-BFGS on top of the running score z:
  fx = z + sum_k g_k(x) h_k(x)
  gate g:   softmax over K-1 free linear logits + an implicit 0 logit   (mlr, sdt)
            or a complete binary tree of K-1 sigmoid nodes, heap indexed (hmlr, hsdt)
  expert h: linear x.v_k (mlr, hmlr) or a scalar leaf value (sdt, hsdt)
Reference: ``J/optimizer/GBMLRHoagOptimizer.java:130-243``, ``GBSDTHoagOptimizer.java:135-240``,
``GBHMLRHoagOptimizer.java:136-253``, ``GBHSDTHoagOptimizer.java:142-250``;
``J/dataflow/GBMLRDataFlow.java`` (z init :115-128, per-tree seed 99999+finished*seed :257,
initW :263-290, continue train :293-538, accumulate :540-587, masks :589-627, dump
``tree-%05d/model-%05d`` + ``tree-info`` :642-748), ``GBSDTDataFlow.java``,
``GBHMLRDataFlow.java``, ``GBHSDTDataFlow.java``; loop ``J/operation/GBMLROperation.java``.

Layouts: mlr/hmlr per feature [gate_0..gate_{K-2} | expert_0..expert_{K-1}] (stride 2K-1);
sdt/hsdt [leaf_0..leaf_{K-1}] + per feature [gate_0..gate_{K-2}] (stride K-1).
Device path: A = X W (gates and experts in one segmented SpMM, J = 2K-1 or K-1),
gate/mixture math as [n, K] tensor ops, G = X^T D (one SpMM).
Reference quirks kept: in random-forest mode the gate gradient uses purefx = fx - z with
fx = mu (z not included), exactly as the reference does.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ...ops._ext import native
from ...utils.errors import YtkLearnError
from ...utils.javafmt import java_double_str, java_float_str
from ..continuous.base import ContinuousModelBase

# loss ids of the fused epilogue (csrc/hip/gbst.hip kLoss*): every scalar loss
GBST_FUSED_MAX_K = 512  # == kGbstWideMax (csrc/hip/gbst.hip)
GBST_LOSS_IDS = {"sigmoid": 0, "l2": 1, "l1": 2, "huber": 3, "poisson": 4, "hinge": 5, "smooth_hinge": 6,
                 "l2_hinge": 7, "exponential": 8, "mape": 9, "smape": 10, "inv_mape": 11}

VARIANTS = {"gbmlr": ("softmax", "linear"), "gbsdt": ("softmax", "scalar"),
            "gbhmlr": ("tree", "linear"), "gbhsdt": ("tree", "scalar")}


def gbst_mixture(A: torch.Tensor, K: int, gate_kind: str, expert_kind: str, leaves: Optional[torch.Tensor]):
    """Mixture pieces from A = X W (fp64 [n, 2K-1] or [n, K-1]).

    Returns (g [n,K] gate probabilities, H [n,K] expert values, mu [n,2K] heap node sums
    (hierarchical gates only, mu[:,1] = sum g*H), sig [n,K-1] node sigmoids or None)."""
    Km1 = K - 1
    logits = A[:, :Km1]
    if expert_kind == "linear":
        H = A[:, Km1:Km1 + K]
    else:
        H = leaves.double()[None, :].expand(A.shape[0], K)
    if gate_kind == "softmax":
        full = torch.cat([logits, torch.zeros_like(logits[:, :1])], dim=1)
        return torch.softmax(full, dim=1), H, None, None
    sig = torch.sigmoid(logits)
    n = A.shape[0]
    prob = torch.ones((n, 2 * K), dtype=torch.float64, device=A.device)  # heap nodes 1..2K-1
    for p in range(1, K):
        prob[:, 2 * p] = prob[:, p] * sig[:, p - 1]          # left child (even heap index): sigma
        prob[:, 2 * p + 1] = prob[:, p] * (1.0 - sig[:, p - 1])
    g = prob[:, K:2 * K]
    mu = torch.zeros((n, 2 * K), dtype=torch.float64, device=A.device)
    mu[:, K:] = g * H
    for p in range(K - 1, 0, -1):
        mu[:, p] = mu[:, 2 * p] + mu[:, 2 * p + 1]
    return g, H, mu, sig


def _jlist(vals) -> str:
    """Java Arrays.toString(double[])."""
    return "[" + ", ".join(java_double_str(float(v)) for v in vals) + "]"


class GBSTModel(ContinuousModelBase):
    def __init__(self, model_name: str, params, data, comm, log, fs=None):
        super().__init__(params, data, comm, log, fs)
        if model_name not in VARIANTS:
            raise YtkLearnError(f"unknown soft tree model {model_name}")
        self.name = model_name
        self.gate_kind, self.expert_kind = VARIANTS[model_name]
        ex = params.extra
        self.K = int(ex.get("k", 16))
        if self.K < 2:
            raise YtkLearnError("soft tree k must be >= 2")
        self.rate = float(ex.get("instance_sample_rate", 1.0))
        self.frate = float(ex.get("feature_sample_rate", 1.0))
        self.tree_num = int(ex.get("tree_num", 1))
        self.type = str(ex.get("type", "gradient_boosting")).lower()
        self.rf = self.type == "random_forest"
        self.lr = 1.0 if self.rf else float(ex.get("learning_rate", 1.0))
        self.leaf_range = [float(v) for v in ex.get("leaf_random_init_range", [-2, 2])]
        base_pred = float(ex.get("uniform_base_prediction", 0.5))
        self.base_score = float(np.float32(self.loss.pred2score(base_pred)))
        self.sample_dep = bool(ex.get("sample_dependent_base_prediction", False))
        self.Km1 = self.K - 1
        if self.expert_kind == "linear":
            self.stride = 2 * self.K - 1
            self.dim = self.F * self.stride
            self.gate_off = 0
        else:
            self.stride = self.K - 1
            self.dim = self.K + self.F * self.stride
            self.gate_off = self.K
        self.L = max(1, math.ceil(math.log2(self.K)))
        self.finished = 0
        dev = self.device
        d = data.train
        self.z = self._init_z(d)
        self.z_test = self._init_z(data.test) if data.test is not None else None
        self.fmask = torch.ones(self.F, dtype=torch.bool, device=dev)
        self.rmask = torch.ones(d.n, dtype=torch.bool, device=dev)
        self.w = torch.zeros(self.dim, dtype=torch.float32, device=dev)
        self.other_train = []
        self.other_test = []
        self.rank = comm.rank if comm is not None else 0

    # ------------------------------------------------------------------ init / masks
    def _init_z(self, d):
        z = torch.full((d.n,), self.base_score, dtype=torch.float32, device=self.device)
        if self.sample_dep and d.init is not None:
            z += self.loss.pred2score(d.init[:, 0].double()).float()
        return z

    def seed(self) -> int:
        s = self.p.random.seed if self.p.random is not None else 111111
        v = 99999 + self.finished * s
        self.log.info(f"new seed:{v}, finished tree num:{self.finished}")
        return v

    def init_w(self):
        rp = self.p.random
        mode = 0 if (rp is None or rp.mode == "normal") else 1
        a, b = ((rp.mean, rp.std) if mode == 0 else (rp.range_start, rp.range_end)) if rp is not None else (0.0, 0.01)
        nat = native()
        w = np.zeros(self.dim, np.float32)
        if self.expert_kind == "linear":
            start = self.stride if self.p.model.need_bias else 0
            w[start:] = nat.java_random_seq(self.seed(), [(mode, self.dim - start, a, b)]).astype(np.float32)
        else:
            v = nat.java_random_seq(self.seed(), [(mode, self.dim, a, b),
                                                 (1, self.K, self.leaf_range[0], self.leaf_range[1])])
            w[:] = v[:self.dim].astype(np.float32)
            w[:self.K] = v[self.dim:].astype(np.float32)
            if self.p.model.need_bias:
                w[self.K:2 * self.K - 1] = 0.0
        self.w.copy_(torch.from_numpy(w))

    def next_sample(self, rate: float, frate: float):
        """Row mask (per-rank seeded: the reference uses an unseeded Random) and the
        globally agreed feature mask (Random(getSeed()).nextDouble() <= rate)."""
        g = torch.Generator(device="cpu")
        g.manual_seed(1234567 + 1000003 * self.rank + 7919 * self.finished)
        self.rmask = (torch.rand(self.data.train.n, generator=g, dtype=torch.float64) <= rate).to(self.device)
        u = native().java_random_seq(self.seed(), [(3, self.F, 0.0, 1.0)])
        fm = u <= frate
        if self.p.model.need_bias:
            fm[0] = True
        self.fmask = torch.from_numpy(fm).to(self.device)

    def regular_groups(self) -> List[Tuple[int, int]]:
        if self.expert_kind == "linear":
            return [(self.stride if self.p.model.need_bias else 0, self.dim)]
        return [(0, self.K), ((2 * self.K - 1) if self.p.model.need_bias else self.K, self.dim)]

    def extra_info(self) -> str:
        return f"[round={self.finished + 1}] "

    # ------------------------------------------------------------------ math
    def _masked_W(self, w, fmask):
        Wf = w[self.gate_off:].view(self.F, self.stride)
        if fmask is None or bool(fmask.all()):
            return Wf
        Wm = Wf.clone()
        Wm[~fmask, :self.Km1] = 0.0
        return Wm

    def _mixture(self, X, w, fmask):
        """(gate probs g [n,K], expert values H [n,K], mu_nodes or None, sig [n,K-1] or None) in fp64."""
        A = X.matmul(self._masked_W(w, fmask).contiguous()).double()
        leaves = w[:self.K] if self.expert_kind == "scalar" else None
        return gbst_mixture(A, self.K, self.gate_kind, self.expert_kind, leaves)

    def _fused_ok(self, X) -> bool:
        """The fused HIP epilogue (csrc/hip/gbst.hip) covers every scalar loss
        (GBST_LOSS_IDS) and 2 <= K <= 512 (softmax and hierarchical gates: lane groups per row
        up to K = 64, one wave per row with several experts per lane above); otherwise
        (K > 512, CPU, YTK_GBST_FUSED=0) the fp64 torch path runs."""
        K = self.K
        return (X.values.is_cuda and self.loss.name in GBST_LOSS_IDS and 2 <= K <= GBST_FUSED_MAX_K
                and os.environ.get("YTK_GBST_FUSED", "1") != "0")

    def _lgamma_y(self, d):
        """lgamma(y + 1) per row, fp64 (poisson's label term, computed once per data set)."""
        cache = self.__dict__.setdefault("_lgy_cache", {})
        key = d.y.data_ptr()
        if key not in cache:
            cache[key] = torch.lgamma(d.y[:, 0].double() + 1.0).contiguous()
        return cache[key]

    def _row_ld(self) -> int:
        """Row pitch (floats) of W, A and D in the fused path: the gate / expert row of
        2K - 1 floats padded to a line multiple (31 -> 32: a 124-B row straddles two 128-B
        lines at 31 of every 32 offsets, so every SpMM gather fetched two lines); the model
        vector keeps its [F][stride] layout (YTK_GBST_PAD=0: unpadded)."""
        J = self.stride
        if os.environ.get("YTK_GBST_PAD", "1") == "0" or J < 6:
            return J
        p = 8
        while p < J and p < 32:
            p <<= 1
        return p if J <= 32 else -(-J // 32) * 32

    def _forward_fused(self, X, d, z, w, g_out, train: bool):
        from ...ops._ext import hip, ptr, stream
        fmask = self.fmask
        J, ld = self.stride, self._row_ld()
        Wm = self._masked_W(w, fmask)
        if ld != J:  # line-aligned rows: W copied into a padded buffer, A and D pitched alike
            Wp = self.__dict__.get("_wpad")
            if Wp is None or Wp.shape != (self.F, ld) or Wp.device != Wm.device:
                Wp = self._wpad = torch.zeros((self.F, ld), dtype=torch.float32, device=Wm.device)
            Wp[:, :J].copy_(Wm)
            A = torch.empty((X.n, ld), dtype=torch.float32, device=Wm.device)[:, :J]
            X.matmul(Wp[:, :J], out=A)  # float32 [n, stride], row pitch ld (segmented SpMM)
        else:
            A = X.matmul(Wm.contiguous())  # float32 [n, stride] (segmented SpMM)
        n, K = A.shape[0], self.K
        acc = torch.zeros(2 + 2 * K, dtype=torch.float64, device=A.device)
        pred = torch.empty(n, dtype=torch.float32, device=A.device)
        want = g_out is not None
        D = torch.empty((n, ld), dtype=torch.float32, device=A.device)[:, :J] if want else None
        y = d.y[:, 0].contiguous()
        wt = d.weight.contiguous()
        mask = self.rmask.view(torch.uint8) if train else None
        leaves = w[:K].contiguous() if self.expert_kind == "scalar" else None
        hip().gbst_epilogue(ptr(A), A.stride(0), ptr(z), ptr(y), ptr(wt), ptr(mask), float(1.0 / self.rate),
                            ptr(leaves), n, K, 1 if self.gate_kind == "tree" else 0,
                            1 if self.expert_kind == "linear" else 0, GBST_LOSS_IDS[self.loss.name],
                            float(getattr(self.loss, "delta", 0.0)), 1 if self.rf else 0, self.finished + 1, 1 if want else 0, ptr(D), ld,
                            ptr(pred), ptr(acc), ptr(self._lgamma_y(d)) if self.loss.name == "poisson" else 0,
                            stream(A))
        if want:
            G = g_out[self.gate_off:].view(self.F, self.stride)
            X.t_matmul(D, out=G)
            if fmask is not None and not bool(fmask.all()):
                G[~fmask, :self.Km1] = 0.0
        a = acc.cpu()
        if want and self.expert_kind == "scalar":
            g_out[:K] = a[2 + K:2 + 2 * K].float().to(g_out.device)
        samples = a[2:2 + K].clone() if train else None
        return float(a[0]), pred, float(a[1]), samples

    def _forward(self, X, d, z, w, g_out, train: bool):
        if self._fused_ok(X):
            return self._forward_fused(X, d, z, w, g_out, train)
        fmask = self.fmask
        gk, H, mu, sig = self._mixture(X, w, fmask)
        purefx_mix = (gk * H).sum(1) if mu is None else mu[:, 1]
        zz = z.double()
        fx = purefx_mix if self.rf else zz + purefx_mix
        y = d.y[:, 0].double()
        wt = d.weight.double()
        if train:
            mask = self.rmask.double()
            wt = wt * mask / self.rate
        lv = self.loss.loss(fx, y)
        loss = float((wt * lv).sum())
        T = self.finished + 1
        if self.rf:
            pred = self.loss.predict((zz + purefx_mix) / T).float()
            rf_loss = float((wt * self.loss.loss((zz + purefx_mix) / T, y)).sum())
        else:
            pred = self.loss.predict(fx).float()
            rf_loss = 0.0
        if train:
            samples = (gk * self.rmask.double()[:, None]).sum(0)
        else:
            samples = None
        if g_out is not None:
            c = wt * self.loss.grad(fx, y)
            purefx = fx - zz  # reference: fx - z (in RF mode fx excludes z)
            n = fx.shape[0]
            D = torch.zeros((n, self.stride), dtype=torch.float64, device=fx.device)
            if self.gate_kind == "softmax":
                D[:, :self.Km1] = c[:, None] * gk[:, :self.Km1] * (H[:, :self.Km1] - purefx[:, None])
            else:
                for p in range(1, self.K):
                    D[:, p - 1] = c * (mu[:, 2 * p] - sig[:, p - 1] * mu[:, p])
            if self.expert_kind == "linear":
                D[:, self.Km1:] = c[:, None] * gk
            G = g_out[self.gate_off:].view(self.F, self.stride)
            X.t_matmul(D.float().contiguous(), out=G)
            if fmask is not None and not bool(fmask.all()):
                G[~fmask, :self.Km1] = 0.0
            if self.expert_kind == "scalar":
                g_out[:self.K] = (c[:, None] * gk).sum(0).float()
        return loss, pred, rf_loss, samples

    def _allreduce_vec(self, t):
        if self.comm is not None and self.comm.is_dist:
            self.comm.allreduce_(t)
        return t

    def pure_loss_grad(self, w, g):
        loss, pred, rf_loss, samples = self._forward(self.X, self.data.train, self.z, w, g, True)
        self.pred = pred[:, None]
        if self.rf:
            t = self._allreduce_vec(torch.tensor([rf_loss], dtype=torch.float64))
            self.other_train.append(f"train loss(random forest):{java_double_str(float(t[0]) / self.data.train.weight_sum)}")
        s = self._allreduce_vec(samples.cpu())
        tot = float(s.sum())
        world = self.comm.world if self.comm is not None else 1
        dist = (s / tot).tolist() if tot > 0 else [0.0] * self.K
        self.other_train.append(f"all samples:{java_double_str(tot)}, ideal avg samples:"
                                f"{java_double_str(tot / world)}, samples distribution:{_jlist(dist)}")
        return loss

    def test_pure_loss_grad(self, w, g):
        if self.data.test is None:
            return 0.0
        if g is not None and self.Xt._csc is None:
            self.Xt._build_csc()
        loss, pred, rf_loss, _ = self._forward(self.Xt, self.data.test, self.z_test, w, g, False)
        self.pred_test = pred[:, None]
        if self.rf:
            t = self._allreduce_vec(torch.tensor([rf_loss], dtype=torch.float64))
            self.other_test.append(f"test loss(random forest):{java_double_str(float(t[0]) / self.data.test.weight_sum)}")
        return loss

    def other_train_info(self) -> str:
        s = "".join(x + "\n" for x in self.other_train)
        self.other_train.clear()
        return s

    def other_test_info(self) -> str:
        s = "".join(x + "\n" for x in self.other_test)
        self.other_test.clear()
        return s

    # ------------------------------------------------------------------ boosting
    def accumulate(self, X, z, w, fmask):
        """z += lr * mixture(x) (GBMLRDataFlow.accumulate)."""
        gk, H, mu, _ = self._mixture(X, w, fmask)
        f = (gk * H).sum(1) if mu is None else mu[:, 1]
        z.add_((self.lr * f).float())

    def tree_dir(self, t: int) -> str:
        return os.path.join(self.p.model.data_path, "tree-%05d" % t)

    def dump(self, w, precision):
        wn = w.detach().cpu().numpy()
        fm = self.fmask.cpu().numpy()
        start, end = self.index_range(self.F)
        delim = self.p.model.delim
        lines = [f"k:{self.K}"]
        if self.expert_kind == "scalar":
            lines.append(delim.join(java_float_str(v) for v in wn[:self.K]))
        Wf = wn[self.gate_off:].reshape(self.F, self.stride)
        dict_lines = []
        bias = self.p.model.need_bias
        for i in range(start, end):
            n = self.data.names[i]
            row = Wf[i].copy()
            if not (bias and i == 0) and not fm[i]:
                row[:self.Km1] = 0.0
            vals = "".join(java_float_str(v) + delim for v in row)
            lines.append(n + delim + vals)
            if not (bias and i == 0):
                dict_lines.append(n)
        rank = self.rank
        mpath = os.path.join(self.tree_dir(self.finished), "model-%05d" % rank)
        dpath = os.path.join(self.p.model.data_path + "_dict", "dict-%05d" % rank)
        with self.fs.open_write(mpath) as f:
            f.write("\n".join(lines) + "\n")
        with self.fs.open_write(dpath) as f:
            f.write("".join(x + "\n" for x in dict_lines))
        self.log.info(f"model is written to {mpath}")
        self.log.info(f"model-dict is written to {dpath}")
        self.dump_info()

    def dump_info(self):
        if self.rank != 0:
            return
        path = os.path.join(self.p.model.data_path, "tree-info")
        self.log.info(f"begin dumping tree info, k:{self.K}, tree_num:{self.tree_num}, finished_tree_num:"
                      f"{self.finished}, uniform_base_prediction:{java_float_str(self.base_score)}")
        with self.fs.open_write(path) as f:
            f.write(f"K:{self.K}\ntree_num:{self.tree_num}\nfinished_tree_num:{self.finished}\n"
                    f"uniform_base_prediction:{java_float_str(self.base_score)}\n")

    def read_tree(self, t: int) -> Optional[np.ndarray]:
        d = self.tree_dir(t)
        if not self.fs.exists(d):
            return None
        w = np.zeros(self.dim, np.float32)
        delim = self.p.model.delim
        for f in sorted(self.fs.recur_get_paths([d])):
            it = iter(self.fs.read_lines(f))
            head = next(it, "")
            if int(head.split(":")[1]) != self.K:
                raise YtkLearnError(f"old model k != config's K = {self.K}")
            if self.expert_kind == "scalar":
                leaf = next(it, "")
                w[:self.K] = [float(v) for v in leaf.strip().split(delim) if v != ""]
            for line in it:
                s = line.strip()
                if not s:
                    continue
                info = [v for v in s.split(delim)]
                idx = self.data.name2idx.get(info[0])
                if idx is None:
                    continue
                vals = [float(v) for v in info[1:] if v != ""]
                off = self.gate_off + idx * self.stride
                w[off:off + self.stride] = vals[:self.stride]
        return w

    def load_or_init(self) -> bool:
        """Continue-train / just-evaluate: replay finished trees. Returns False when training is done."""
        info_path = os.path.join(self.p.model.data_path, "tree-info")
        want = self.p.model.continue_train or self.p.loss.just_evaluate
        if not want or not self.fs.exists(info_path):
            if want:
                self.log.info("have no model info data, old model doesn't exist, new model..." + info_path)
            self.init_w()
            self.next_sample(self.rate, self.frate)
            return True
        lines = [l.strip() for l in self.fs.read_lines(info_path) if l.strip()]
        if len(lines) != 4:
            raise YtkLearnError("model info must have 4 lines!")
        old_k = int(lines[0].split(":")[1])
        old_trees = int(lines[1].split(":")[1])
        self.finished = int(lines[2].split(":")[1])
        old_base = float(lines[3].split(":")[1])
        if old_k != self.K:
            raise YtkLearnError(f"model info K != config K, model info K:{old_k}, config K:{self.K}")
        if old_trees != self.tree_num:
            self.log.info(f"[WARNING] old tree num:{old_trees} != tree num:{self.tree_num}")
        if self.finished >= self.tree_num and not self.p.loss.just_evaluate:
            self.log.info(f"finished tree num:{self.finished} >= tree num:{self.tree_num}, finished directly!")
            return False
        if abs(old_base - self.base_score) > 1e-6:
            raise YtkLearnError(f"old uniform_base_prediction != uniform_base_prediction, old:{old_base}, "
                                f"new:{self.base_score}")
        ones = torch.ones(self.F, dtype=torch.bool, device=self.device)
        for t in range(self.finished):
            wt = self.read_tree(t)
            if wt is None:
                raise YtkLearnError(f"finished tree {t} missing under {self.p.model.data_path}")
            wdev = torch.from_numpy(wt).to(self.device)
            self.accumulate(self.X, self.z, wdev, ones)
            if self.Xt is not None:
                self.accumulate(self.Xt, self.z_test, wdev, ones)
        if self.p.loss.just_evaluate:
            self.next_sample(1.0, 1.0)
            return True
        cur = self.read_tree(self.finished)
        self.next_sample(self.rate, self.frate)
        if cur is None:
            self.log.info("unfinished tree not exited!")
            self.init_w()
        else:
            self.log.info("unfinished tree existed! will be readed ...")
            self.w.copy_(torch.from_numpy(cur))
        return True
