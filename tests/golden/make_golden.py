"""Generate the golden fixtures under tests/golden/ from the CPU oracle (REF-R).

    python tests/golden/make_golden.py            # all fixtures
    python tests/golden/make_golden.py e2e_c1     # one

PARITY UNPINNED: the reference ships no golden vectors and could not be imported here
(SURVEY.md 8(c)), so these fixtures are the oracle's outputs, recorded with the torch
version / CPU capability that produced them.  The oracle itself is pinned by the hand KATs
in tests/test_oracle_kat.py.  Inputs use seeded random floats and dyadic grids (coordinates
k/64, exactly representable, so BLAS/FMA ordering cannot change any distance).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deepvcp-pointcloud-registration_amd"))

import oracle as O  # noqa: E402
from dvcp.synthetic import condition_weights, make_pairs, randomize_bn  # noqa: E402

META = dict(torch=torch.__version__, cpu=torch.backends.cpu.get_cpu_capability())


def save(name, **arrays):
    arrays = {k: (v.numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in arrays.items()}
    arrays["meta"] = np.array(repr(META))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    print("wrote", name, sum(a.nbytes for a in arrays.values()) // 1024, "KiB raw")


def dyadic(shape, lim, seed, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    return (torch.randint(-lim, lim + 1, shape, generator=g).to(torch.float64) / 64.0).to(dtype)


def weights_dict(model):
    return {"w::" + k: v.detach().clone() for k, v in model.state_dict().items()}


# ---------------------------------------------------------------------------------------------
def gen_fps():
    g = torch.Generator().manual_seed(11)
    xyz = torch.rand(2, 2048, 3, generator=g) * 2 - 1
    start = torch.tensor([5, 2047])
    save("fps_f32", xyz=xyz, start=start, npoint=np.int64(512), idx=O.farthest_point_sample(xyz, 512, start))
    xyz = dyadic((2, 1024, 3), 8, 12)  # heavy duplicates and equal distances: tie-break paths
    start = torch.tensor([0, 77])
    save("fps_dyadic", xyz=xyz, start=start, npoint=np.int64(1500),
         idx=O.farthest_point_sample(xyz, 1500, start))
    x64 = torch.rand(2, 1500, 3, generator=g, dtype=torch.float64) * 2 - 1
    start = torch.tensor([3, 1499])
    save("fps_f64", xyz=x64, start=start, npoint=np.int64(700), idx=O.farthest_point_sample(x64, 700, start))


def gen_ball():
    g = torch.Generator().manual_seed(21)
    xyz = torch.rand(2, 2048, 3, generator=g) * 2 - 1
    ctr = xyz[:, torch.randperm(2048, generator=g)[:300], :]
    out = {}
    for r, ns in ((0.1, 256), (0.2, 128), (0.4, 64)):
        out[f"idx_{ns}"] = O.query_ball_point(r, ns, xyz, ctr)
    save("ball_f32", xyz=xyz, ctr=ctr, **out)
    # dyadic: many points exactly on the sphere |p - c| = r (r = 0.25 = 16/64)
    xyz = dyadic((2, 1500, 3), 24, 22)
    ctr = dyadic((2, 200, 3), 24, 23)
    save("ball_dyadic", xyz=xyz, ctr=ctr, idx_32=O.query_ball_point(0.25, 32, xyz, ctr),
         idx_200=O.query_ball_point(0.25, 200, xyz, ctr))
    x64 = torch.rand(1, 1200, 3, generator=g, dtype=torch.float64) * 2 - 1
    c64 = x64[:, :400, :]
    save("ball_f64", xyz=x64, ctr=c64, idx_128=O.query_ball_point(0.2, 128, x64, c64))


def gen_knn():
    g = torch.Generator().manual_seed(31)
    ref = torch.rand(2, 1000, 3, generator=g) * 2 - 1
    qry = torch.rand(2, 3000, 3, generator=g) * 3 - 1.5
    d, i = O.KNN(k=32, transpose_mode=True)(ref, qry)
    save("knn_f32", ref=ref, qry=qry, dist=d, idx=i)
    ref = dyadic((2, 600, 3), 6, 32)     # equidistant references everywhere
    qry = dyadic((2, 500, 3), 6, 33)
    d, i = O.KNN(k=32, transpose_mode=True)(ref, qry)
    save("knn_dyadic", ref=ref, qry=qry, dist=d, idx=i)
    d1, i1 = O.KNN(k=1, transpose_mode=False)(ref.transpose(1, 2), qry.transpose(1, 2))
    save("knn_k1", ref=ref, qry=qry, dist=d1, idx=i1)


def gen_voxel():
    g = torch.Generator().manual_seed(41)
    pts = (torch.rand(2, 6, 3, generator=g, dtype=torch.float64) * 20 - 10)
    pts[0, 0] = 0.0
    save("voxel", pts=pts, cand_r2=O.voxelize(pts, 2.0, 0.4), cand_r1=O.voxelize(pts, 1.0, 0.4))


def gen_rigid():
    g = torch.Generator().manual_seed(51)
    B, n = 3, 64
    x = torch.rand(B, n, 3, generator=g, dtype=torch.float64) * 2 - 1
    _, _, Rt, tt = make_pairs(B, 8, seed=52)
    y = (Rt @ x.transpose(1, 2) + tt).transpose(1, 2) + 0.05 * torch.randn(B, n, 3, generator=g, dtype=torch.float64)
    y = y.float()
    loss, R, t = O.deepVCP_loss(x, y, Rt, tt, 0.5)
    R1, t1 = O.get_rigid_transform(x.transpose(1, 2).contiguous(), y.double().transpose(1, 2).contiguous())
    save("rigid", x=x, y=y, R_true=Rt, t_true=tt, loss=loss, R=R, t=t, R1=R1, t1=t1)


def _e2e(name, B, N, normals, K, r, s, fe_npoint, seed):
    src, tgt, R, t = make_pairs(B, N, normals=normals, seed=seed)
    torch.manual_seed(0)
    model = O.DeepVCP(use_normal=normals, K=K, r=r, s=s, fe_npoint=fe_npoint).eval()
    randomize_bn(model)
    with torch.no_grad():
        _, calib = model.FE1(src)          # conditioned WL (dvcp.synthetic.condition_weights)
    condition_weights(model, feats=calib)
    torch.manual_seed(1)
    sizes = (N, fe_npoint, fe_npoint, K, N, fe_npoint, fe_npoint)
    starts = torch.stack([torch.randint(0, n, (B,), dtype=torch.long) for n in sizes])
    torch.manual_seed(1)  # the oracle draws the same starts itself
    with torch.no_grad(), O.tracing() as tr:
        kp, vcp = model(src, tgt, R, torch.zeros(1, 3))
        loss, Rp, tp = O.deepVCP_loss(kp, vcp, R, t, 0.5)
    names = [n for n, _ in tr]
    pick = {}
    fps_i = [v for n, v in tr if n == "fps_idx"]
    pick["fps_src"] = torch.stack(fps_i[0:3])
    pick["fps_kp"] = fps_i[3]
    pick["fps_tgt"] = torch.stack(fps_i[4:7])
    fe_x = [v for n, v in tr if n == "fe_xyz"]
    fe_f = [v for n, v in tr if n == "fe_feat"]
    pick["fe_xyz_src"], pick["fe_xyz_tgt"] = fe_x
    pick["fe_feat_src"], pick["fe_feat_tgt"] = fe_f
    d = dict(tr)
    pick["score"] = d["wl_score"][..., 0]
    pick["topk"] = d["topk_idx"]
    pick["keypts"] = d["keypts"]
    pick["src_cat"] = d["src_cat"]
    pick["moved"] = d["moved"]
    pick["src_dfe"] = d["src_dfe"]
    nq = 4096
    pick["knn_idx_head"] = d["knn_idx"][:, :nq].int()
    pick["knn_dist_head"] = d["knn_dist"][:, :nq]
    pick["tgt_dfe_head"] = d["tgt_dfe"].reshape(B, -1, 32)[:, :nq]
    pick["cpg_weight"] = d["cpg_weight"]
    save(name, src=src, tgt=tgt, R_gt=R, t_gt=t, starts=starts, K=np.int64(K), r=np.float64(r), s=np.float64(s),
         fe_npoint=np.int64(fe_npoint), normals=np.bool_(normals), keypts_out=kp, vcp=vcp, loss=loss, R=Rp, t=tp,
         trace_names=np.array(names), **pick, **weights_dict(model))


def gen_e2e_small():
    _e2e("e2e_c3small", B=2, N=2048, normals=False, K=64, r=2.0, s=0.4, fe_npoint=512, seed=1234)


def gen_e2e_c1():
    # literal config C1: ModelNet-like, B=1, N=1024, xyz+normals fp64, K=64, r=1.0, npoint 10000
    _e2e("e2e_c1", B=1, N=1024, normals=True, K=64, r=1.0, s=0.4, fe_npoint=10000, seed=4321)


GENS = dict(fps=gen_fps, ball=gen_ball, knn=gen_knn, voxel=gen_voxel, rigid=gen_rigid, e2e_small=gen_e2e_small,
            e2e_c1=gen_e2e_c1)

if __name__ == "__main__":
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    which = sys.argv[1:] or list(GENS)
    for w in which:
        GENS[w]()
