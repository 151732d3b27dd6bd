import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from ytk_learn_amd.ops import gbdt as gops
cuda = torch.device("cuda", 0)
SG, SH = gops.fixed_point_scales(3.0, 0.25, 200000)
def run(F, nb, N, ips, slot_ids, mode):
    g = torch.Generator().manual_seed(5)
    stride = ((F + 31) // 32) * 32
    bins = torch.zeros((N, stride), dtype=torch.uint8); bins[:, :F] = torch.randint(0, nb, (N, F), generator=g).to(torch.uint8)
    gh = torch.empty((N, 2)); gh[:, 0] = torch.randn(N, generator=g); gh[:, 1] = torch.rand(N, generator=g) * 0.25
    B = ((nb + 3) // 4) * 4
    perm = torch.randperm(N, generator=g).to(torch.int32)
    nslot = len(slot_ids)
    edges = np.linspace(0, N, nslot * ips + 1).astype(np.int64)
    work = np.array([(slot_ids[k // ips], edges[k], edges[k + 1], 0) for k in range(nslot * ips)], np.int32)
    wt = torch.from_numpy(work)
    hc = torch.zeros((6, B, F, 2), dtype=torch.int64)
    gops.hist_build(bins, F, gh, perm, wt, hc, B, SG, SH)
    hg = torch.zeros((6, B, F, 2), dtype=torch.int64, device=cuda)
    st = torch.empty(len(work) * ((F + 31) // 32) * B * 64, dtype=torch.int64, device=cuda)
    sid = torch.tensor(slot_ids, dtype=torch.int32, device=cuda)
    contiguous = slot_ids == list(range(slot_ids[0], slot_ids[0] + nslot))
    if mode == "staged":
        gops.hist_build(bins.to(cuda), F, gh.to(cuda), perm.to(cuda), wt.to(cuda), hg, B, SG, SH, staging=st,
                        slot_base=slot_ids[0], nslots=nslot, slot_ids=None if contiguous else sid)
    else:
        gops.hist_build(bins.to(cuda), F, gh.to(cuda), perm.to(cuda), wt.to(cuda), hg, B, SG, SH)
    hg = hg.cpu()
    bad = [(s, int((hg[s] != hc[s]).sum()), int((hc[s] != 0).sum())) for s in range(6)]
    print(mode, F, nb, N, ips, slot_ids, "contig" if contiguous else "ids", bad, flush=True)
for mode in ("plain", "staged"):
    for ips in (1, 2, 8, 33):
        run(28, 255, 200000, ips, [2, 3, 4], mode)
