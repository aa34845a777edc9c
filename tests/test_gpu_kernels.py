"""GPU parity of every HIP kernel against the oracle (golden fixtures + live, seeded).

Bars: bit-exact for indices (FPS, ball query, kNN, top-k, candidate grid) and kNN distances;
fp32 feature stages within rtol 1e-5 / atol 1e-5 of the oracle's torch CPU ops (different fp32
summation order); fp64 pose solve within 1e-9.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def T(a, dev=None):
    t = torch.from_numpy(np.asarray(a))
    return t.to(dev) if dev is not None else t


def ball_mismatch_ok(xyz, ctr, got, want, radius, ulps=4):
    """Rows that differ may only differ by points whose d2 sits within `ulps` of radius^2."""
    import oracle as O
    bad = (got != want).any(-1)
    if not bad.any():
        return True
    d2 = O.square_distance(ctr, xyz)
    r2 = torch.tensor(radius ** 2, dtype=xyz.dtype)
    tol = ulps * torch.finfo(xyz.dtype).eps * float(r2)
    for b, s in bad.nonzero().tolist():
        a, w = set(got[b, s].tolist()), set(want[b, s].tolist())
        for n in a ^ w:
            if n < xyz.shape[1] and abs(float(d2[b, s, n]) - float(r2)) > tol:
                return False
    return True


# ---------------------------------------------------------------------------------------- FPS
@pytest.mark.parametrize("name", ["fps_f32", "fps_dyadic", "fps_f64"])
def test_fps_golden(cuda, name):
    import dvcp.pointnet2_utils as P
    from dvcp import ops
    z = golden(name)
    xyz = T(z["xyz"], cuda)
    idx = P.farthest_point_sample(xyz, int(z["npoint"]), start=T(z["start"]))
    assert torch.equal(idx.cpu(), T(z["idx"]))
    # channel-first layout + sampled centres
    idx2, ctr = ops.fps(xyz.transpose(1, 2).contiguous(), int(z["npoint"]), T(z["start"], cuda), pdim=2)
    assert torch.equal(idx2, idx)
    gathered = torch.stack([xyz[b, idx[b]] for b in range(xyz.shape[0])]).transpose(1, 2)
    assert torch.equal(ctr, gathered)


def test_fps_live_vs_oracle(cuda):
    import oracle as O
    import dvcp.pointnet2_utils as P
    g = torch.Generator().manual_seed(101)
    for N, npoint in ((16384, 2000), (10000, 10000), (333, 1000), (5, 7)):
        xyz = torch.rand(2, N, 3, generator=g) * 2 - 1
        start = torch.randint(0, N, (2,), generator=g)
        want = O.farthest_point_sample(xyz, npoint, start)
        got = P.farthest_point_sample(xyz.to(cuda), npoint, start=start).cpu()
        assert torch.equal(got, want), (N, npoint)


@pytest.mark.parametrize("case", ["dyadic", "duplicates", "surface", "npoint_gt_n", "f64"])
def test_fps_select_vs_oracle(cuda, case):
    """The threshold-select kernel (N >= 2048) on inputs that stress its exactness argument:
    equal running minima everywhere (dyadic grid: the one-argmax fallback), exact duplicate
    points, a 2-D surface, npoint > N (all minima reach 0), and fp64 coordinates."""
    import oracle as O
    import dvcp.pointnet2_utils as P
    g = torch.Generator().manual_seed(["dyadic", "duplicates", "surface", "npoint_gt_n", "f64"].index(case) + 200)
    N, npoint, dt = 4096, 1500, torch.float32
    if case == "dyadic":
        xyz = torch.randint(-8, 9, (2, N, 3), generator=g).float() / 8
    elif case == "duplicates":
        xyz = (torch.rand(2, N // 4, 3, generator=g) * 2 - 1).repeat_interleave(4, dim=1)
    elif case == "surface":
        v = torch.randn(2, N, 3, generator=g)
        xyz = v / v.norm(dim=2, keepdim=True)
    elif case == "npoint_gt_n":
        N, npoint = 2100, 2600
        xyz = torch.rand(2, N, 3, generator=g) * 2 - 1
    else:
        dt = torch.float64
        xyz = torch.rand(2, N, 3, generator=g, dtype=dt) * 2 - 1
    start = torch.randint(0, N, (2,), generator=g)
    want = O.farthest_point_sample(xyz, npoint, start)
    got = P.farthest_point_sample(xyz.to(cuda), npoint, start=start).cpu()
    assert torch.equal(got, want), (case, int((got != want).nonzero()[0, 1]) if (got != want).any() else -1)


def _split_cloud(case, g, B=2):
    N, npoint = 4096, 1500
    if case == "dyadic":
        xyz = torch.randint(-8, 9, (B, N, 3), generator=g).float() / 8
    elif case == "duplicates":
        xyz = (torch.rand(B, N // 4, 3, generator=g) * 2 - 1).repeat_interleave(4, dim=1)
    elif case == "surface":
        v = torch.randn(B, N, 3, generator=g)
        xyz = v / v.norm(dim=2, keepdim=True)
    elif case == "npoint_gt_n":
        N, npoint = 3000, 3600
        xyz = torch.rand(B, N, 3, generator=g) * 2 - 1
    elif case == "full_perm":  # sa2 / sa3 of C3: every point picked, parts run empty near the end
        N, npoint = 10000, 10000
        xyz = torch.rand(B, N, 3, generator=g) * 2 - 1
    elif case == "clustered":  # one dense blob and a sparse halo: the parts' maxima differ widely
        xyz = torch.cat([torch.randn(B, N // 2, 3, generator=g) * 0.02,
                         torch.rand(B, N - N // 2, 3, generator=g) * 2 - 1], 1)
        xyz = xyz[:, torch.randperm(N, generator=g)]
    else:
        xyz = torch.rand(B, N, 3, generator=g) * 2 - 1
    return xyz, npoint


@pytest.mark.parametrize("parts", [2, 4, 8])
@pytest.mark.parametrize("case", ["generic", "dyadic", "duplicates", "surface", "npoint_gt_n", "full_perm",
                                  "clustered"])
def test_fps_split_select_vs_oracle(cuda, parts, case):
    """The split select (round 6: S workgroups per cloud, one candidate-list exchange per round)
    against the oracle, bit for bit, on the inputs that stress the select kernel's exactness
    argument -- equal minima everywhere (the per-part fallback and the global argmax round),
    duplicates (minima reaching 0), npoint > N and a full permutation (parts whose points are all
    at 0: "empty"), a surface, and a clustered cloud whose parts' values differ widely."""
    import oracle as O
    from dvcp import ops
    g = torch.Generator().manual_seed(500 + 7 * parts + ["generic", "dyadic", "duplicates", "surface", "npoint_gt_n",
                                                         "full_perm", "clustered"].index(case))
    xyz, npoint = _split_cloud(case, g)
    N = xyz.shape[1]
    start = torch.randint(0, N, (xyz.shape[0],), generator=g)
    want = O.farthest_point_sample(xyz, npoint, start)
    got, ctr = ops.fps(xyz.to(cuda), npoint, start.to(cuda), pdim=1, parts=parts)
    got = got.cpu()
    assert torch.equal(got, want), (case, parts, int((got != want).nonzero()[0, 1]) if (got != want).any() else -1)
    gathered = torch.stack([xyz[b, want[b]] for b in range(xyz.shape[0])]).transpose(1, 2)
    assert torch.equal(ctr.cpu(), gathered)


@pytest.mark.parametrize("N", [16384, 10000])
def test_fps_split_select_c3_equals_one_workgroup(cuda, N):
    """C3's FE chain sizes, 16 clouds as one launch (the bench's batch): the split select at 2, 4
    and 8 workgroups per cloud returns the one-workgroup kernel's indices (itself bit-exact
    against the oracle: test_fps_live_vs_oracle, test_e2e_c3_pair_vs_oracle)."""
    from dvcp import ops
    g = torch.Generator().manual_seed(520 + N % 13)
    xyz = (torch.rand(16, 3, N, generator=g) * 2 - 1).to(cuda)
    start = torch.randint(0, N, (16,), generator=g).to(cuda)
    want, cw = ops.fps(xyz, 10000, start, pdim=2, parts=1)
    for parts in (2, 4, 8):
        got, cg = ops.fps(xyz, 10000, start, pdim=2, parts=parts)
        assert torch.equal(got, want), (parts, int((got != want).nonzero()[0, 1]))
        assert torch.equal(cg, cw)


@pytest.mark.parametrize("N,parts", [(65536, 8), (40000, 8), (32768, 4), (20000, 2)])
def test_fps_split_select_large_clouds(cuda, N, parts):
    """Above the one-workgroup kernel's 16384 points (C5's layer 1 is 65536 -> 10000) the split
    select is the default: part 0 sorts the whole cloud into the workspace and each part reads its
    own groups' indices.  Against the oracle on a prefix, and against the per-step split kernel
    (parts=1) on the C5 chain length, bit for bit."""
    import oracle as O
    from dvcp import ops
    g = torch.Generator().manual_seed(540 + N % 97)
    xyz = torch.rand(2, N, 3, generator=g) * 2 - 1
    start = torch.randint(0, N, (2,), generator=g)
    want = O.farthest_point_sample(xyz, 1500, start)
    got, ctr = ops.fps(xyz.to(cuda), 1500, start.to(cuda), pdim=1, parts=parts)
    assert torch.equal(got.cpu(), want), int((got.cpu() != want).nonzero()[0, 1])
    gathered = torch.stack([xyz[b, want[b]] for b in range(2)]).transpose(1, 2)
    assert torch.equal(ctr.cpu(), gathered)
    xt = xyz.transpose(1, 2).contiguous().to(cuda)
    ref, cref = ops.fps(xt, 10000, start.to(cuda), pdim=2, parts=1)
    got, cgot = ops.fps(xt, 10000, start.to(cuda), pdim=2)  # the default: 8 parts above 16384 points
    assert torch.equal(got, ref), int((got != ref).nonzero()[0, 1])
    assert torch.equal(cgot, cref)
    if parts != 8:
        got, _ = ops.fps(xt, 10000, start.to(cuda), pdim=2, parts=parts)
        assert torch.equal(got, ref), int((got != ref).nonzero()[0, 1])


@pytest.mark.parametrize("case", ["duplicates", "clustered", "dyadic"])
def test_fps_split_select_large_cloud_edge_cases(cuda, case):
    """The large-cloud split select (8 parts, 32768 points) on the inputs that stress the select's
    exactness argument: repeated points (minima reaching 0, parts running empty), a dense blob in a
    sparse halo, and a dyadic grid of equal minima (ties to the lowest index), against the oracle."""
    import oracle as O
    from dvcp import ops
    g = torch.Generator().manual_seed(560 + ["duplicates", "clustered", "dyadic"].index(case))
    B, N = 2, 32768
    if case == "duplicates":
        xyz = (torch.rand(B, N // 8, 3, generator=g) * 2 - 1).repeat_interleave(8, dim=1)
        npoint = 5000   # beyond the 4096 distinct points: the chain continues at minimum 0
    elif case == "clustered":
        xyz = torch.cat([torch.randn(B, N // 2, 3, generator=g) * 0.02,
                         torch.rand(B, N - N // 2, 3, generator=g) * 2 - 1], 1)
        xyz = xyz[:, torch.randperm(N, generator=g)]
        npoint = 2000
    else:
        xyz = torch.randint(-16, 17, (B, N, 3), generator=g).float() / 16
        npoint = 2000
    start = torch.randint(0, N, (B,), generator=g)
    want = O.farthest_point_sample(xyz, npoint, start)
    got, _ = ops.fps(xyz.to(cuda), npoint, start.to(cuda), pdim=1)
    got = got.cpu()
    assert torch.equal(got, want), (case, int((got != want).nonzero()[0, 1]) if (got != want).any() else -1)


def test_fps_split_select_large_clouds_many_launches_in_flight(cuda):
    """Ten launches of the large-cloud split select (4 clouds x 8 parts each: 320 full-CU
    workgroups, more than the chip holds at once) on ten streams: roles by start ticket, so every
    waiting workgroup's peers run or come next; the guard word stays clear and every launch equals
    the per-step split kernel's indices."""
    from dvcp import _lib, ops
    g = torch.Generator().manual_seed(570)
    N = 40000
    xyz = (torch.rand(4, 3, N, generator=g) * 2 - 1).to(cuda)
    starts = [torch.randint(0, N, (4,), generator=g).to(cuda) for _ in range(10)]
    streams = [torch.cuda.Stream() for _ in starts]
    outs = []
    for st, s in zip(streams, starts):
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            outs.append(ops.fps(xyz, 3000, s, pdim=2)[0])
    for st in streams:
        torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    _lib.check_device_flags(block=True)
    for s, got in zip(starts, outs):
        want, _ = ops.fps(xyz, 3000, s, pdim=2, parts=1)
        assert torch.equal(got, want)


def test_fps_split_select_many_launches_in_flight(cuda):
    """Ten split-select launches of 16 clouds on ten streams at once (more workgroups than the
    chip holds beside each other): every cloud's workgroups find their peers, the guard word stays
    clear, and each launch equals the one-workgroup kernel."""
    from dvcp import _lib, ops
    g = torch.Generator().manual_seed(530)
    xyz = (torch.rand(16, 3, 16384, generator=g) * 2 - 1).to(cuda)
    starts = [torch.randint(0, 16384, (16,), generator=g).to(cuda) for _ in range(10)]
    streams = [torch.cuda.Stream() for _ in starts]
    outs = []
    for st, s in zip(streams, starts):
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            outs.append(ops.fps(xyz, 4000, s, pdim=2, parts=4)[0])
    for st in streams:
        torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    _lib.check_device_flags(block=True)
    for s, got in zip(starts, outs):
        want, _ = ops.fps(xyz, 4000, s, pdim=2, parts=1)
        assert torch.equal(got, want)


def test_fps_full_size_property(cuda):
    """C3 scale: 16384 -> 10000; the min-distance of each newly picked point to the already
    picked set never increases (the defining FPS invariant), and no index repeats."""
    from dvcp import ops
    g = torch.Generator().manual_seed(102)
    xyz = (torch.rand(4, 16384, 3, generator=g) * 2 - 1).to(cuda)
    idx, _ = ops.fps(xyz, 10000, torch.tensor([0, 1, 16383, 7]).to(cuda), pdim=1)
    for b in range(4):
        assert idx[b].unique().numel() == 10000
        sel = xyz[b, idx[b]].double()
        dmin = torch.full((16384,), float("inf"), dtype=torch.float64, device=cuda)
        prev = []
        x64 = xyz[b].double()
        for i in range(0, 400):
            p = sel[i]
            if i > 0:
                prev.append(float(dmin[idx[b, i]]))
            dmin = torch.minimum(dmin, ((x64 - p) ** 2).sum(-1))
        prev = torch.tensor(prev)
        assert (prev[1:] <= prev[:-1] * (1 + 1e-6) + 1e-12).all()


def _fps_pair_vs_serial(cuda, xyz_cf, s2, s3):
    """ops.fps_pair against the two serial launches it replaces (bit-exact indices and centres)."""
    from dvcp import ops
    N = xyz_cf.shape[2]
    i2, c2, i3, c3 = ops.fps_pair(xyz_cf, s2, s3, pdim=2)
    w2, d2 = ops.fps(xyz_cf, N, s2, pdim=2)
    w3, d3 = ops.fps(d2, N, s3, pdim=2)
    assert torch.equal(i2, w2) and torch.equal(c2, d2)
    assert torch.equal(i3, w3), int((i3 != w3).nonzero()[0, 1])
    assert torch.equal(c3, d3)


@pytest.mark.parametrize("N", [10000, 4096, 2048, 16384])
def test_fps_pair_matches_serial(cuda, N):
    """The paired layer-2/3 launch (layer 3 beside layer 2, from layer 2's pick number start3) on
    generic clouds, with start3 at both ends of the chain and in between."""
    g = torch.Generator().manual_seed(400 + N % 97)
    B = 6
    xyz = (torch.rand(B, 3, N, generator=g) * 2 - 1).to(cuda)
    s2 = torch.randint(0, N, (B,), generator=g)
    s3 = torch.tensor([0, N - 1, 1, N // 2, 37, N - 2])
    _fps_pair_vs_serial(cuda, xyz, s2.to(cuda), s3.to(cuda))


@pytest.mark.parametrize("case", ["dyadic", "duplicates", "mixed", "symmetric"])
def test_fps_pair_ties(cuda, case):
    """Layer-3 argmax ties.  "symmetric": a point-symmetric cloud (p and -p, plus the origin) with
    both layers started at the origin (start3 = 0 picks layer 2's start), so nearly every step
    ties a mirrored pair: the tie groups are reordered by layer 2's pick numbers, or ranked by
    them in the round.  Equal minima everywhere (dyadic grid) and duplicate points (minima
    reaching 0) take the gated serial recomputation; "mixed" puts such clouds beside generic ones
    in one launch.  Every case: the serial launches' result."""
    g = torch.Generator().manual_seed({"dyadic": 410, "duplicates": 411, "mixed": 412, "symmetric": 413}[case])
    B, N = 4, 4096
    if case == "symmetric":
        half = torch.rand(B, 3, 2048, generator=g) * 2 - 1
        xyz = torch.cat([torch.zeros(B, 3, 1), half, -half], 2)[:, :, torch.randperm(4097, generator=g)]
        s2 = torch.stack([int((xyz[b] == 0).all(0).nonzero()[0]) * torch.ones((), dtype=torch.long)
                          for b in range(B)])
        _fps_pair_vs_serial(cuda, xyz.to(cuda), s2.to(cuda), torch.zeros(B, dtype=torch.long).to(cuda))
        return
    if case == "dyadic":
        xyz = torch.randint(-8, 9, (B, 3, N), generator=g).float() / 8
    elif case == "duplicates":
        xyz = (torch.rand(B, 3, N // 4, generator=g) * 2 - 1).repeat_interleave(4, dim=2)
    else:
        xyz = torch.rand(B, 3, N, generator=g) * 2 - 1
        xyz[1] = torch.randint(-8, 9, (3, N), generator=g).float() / 8
        xyz[3, :, N // 2:] = xyz[3, :, :N // 2]
    s2 = torch.randint(0, N, (B,), generator=g)
    s3 = torch.randint(0, N, (B,), generator=g)
    _fps_pair_vs_serial(cuda, xyz.to(cuda), s2.to(cuda), s3.to(cuda))


def test_fps_pair_many_clouds_in_flight(cuda):
    """A C3-sized paired launch (2 x 16 clouds of 10000 points) next to independent work on other
    streams: every layer-3 workgroup waits only for its own cloud's layer-2 workgroup."""
    from dvcp import ops
    g = torch.Generator().manual_seed(420)
    B, N = 16, 10000
    xyz = (torch.rand(B, 3, N, generator=g) * 2 - 1).to(cuda)
    s2 = torch.randint(0, N, (B,), generator=g).to(cuda)
    s3 = torch.randint(0, N, (B,), generator=g).to(cuda)
    other = [torch.cuda.Stream() for _ in range(3)]
    outs = []
    for k, st in enumerate(other):
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            outs.append(ops.fps_pair(xyz, s2, torch.roll(s3, k), pdim=2))
    for st in other:
        torch.cuda.current_stream().wait_stream(st)
    for k, (i2, c2, i3, c3) in enumerate(outs):
        w2, d2 = ops.fps(xyz, N, s2, pdim=2)
        w3, d3 = ops.fps(d2, N, torch.roll(s3, k), pdim=2)
        assert torch.equal(i2, w2) and torch.equal(i3, w3) and torch.equal(c3, d3)


# --------------------------------------------------------------------------------- ball query
@pytest.mark.parametrize("name,radii", [("ball_f32", [(0.1, 256), (0.2, 128), (0.4, 64)]),
                                         ("ball_dyadic", [(0.25, 32), (0.25, 200)]),
                                         ("ball_f64", [(0.2, 128)])])
def test_ball_query_golden(cuda, name, radii):
    import dvcp.pointnet2_utils as P
    z = golden(name)
    xyz, ctr = T(z["xyz"]), T(z["ctr"])
    for r, ns in radii:
        got = P.query_ball_point(r, ns, xyz.to(cuda), ctr.to(cuda)).cpu()
        want = T(z[f"idx_{ns}"])
        if "dyadic" in name:
            assert torch.equal(got, want)
        else:
            assert ball_mismatch_ok(xyz, ctr, got, want, r)


def test_ball_query_compact_matches_padded(cuda):
    from dvcp import ops
    g = torch.Generator().manual_seed(103)
    xyz = (torch.rand(2, 5000, 3, generator=g) * 2 - 1).to(cuda)
    ctr = xyz[:, :700].contiguous()
    cnt, lst, pad = ops.ball_query(xyz, ctr, 0.2, 128, padded=True)
    for b in range(2):
        for s in range(0, 700, 37):
            c = int(cnt[b, s])
            assert 1 <= c <= 128
            hits = lst[b, s, :c].long()
            assert torch.equal(pad[b, s, :c], hits)
            assert (pad[b, s, c:] == hits[0]).all()
            assert (hits[1:] > hits[:-1]).all()


def test_ball_query_no_hit_pads_with_N(cuda):
    import dvcp.pointnet2_utils as P
    xyz = torch.zeros(1, 10, 3, device=cuda)
    ctr = torch.full((1, 2, 3), 5.0, device=cuda)
    assert (P.query_ball_point(0.5, 4, xyz, ctr) == 10).all()


@pytest.mark.parametrize("dtype,N", [(torch.float32, 3000), (torch.float32, 70000), (torch.float64, 3000)])
def test_ball_query_no_hit_compact_row(cuda, dtype, N):
    """The compact output of a centre without hits: count 0 and a valid first list entry (point 0),
    so consumers that clamp count to >= 1 read in bounds; every path (tiled, streaming above 65536
    points, fp64)."""
    from dvcp import ops
    g = torch.Generator().manual_seed(109)
    xyz = (torch.rand(2, 3, N, generator=g, dtype=torch.float64) * 2 - 1).to(dtype).to(cuda)
    ctr = xyz[:, :, :40].clone()
    ctr[:, :, ::3] = 50.0  # every third centre far from every point
    count, lst, _ = ops.ball_query(xyz, ctr.contiguous(), 0.2, 16, pdim=2, cdim_pts=2)
    far = torch.zeros(2, 40, dtype=torch.bool, device=cuda)
    far[:, ::3] = True
    assert (count[far] == 0).all() and (count[~far] >= 1).all()
    assert (lst[far][:, 0] == 0).all()


def _bq_case(case, g):
    """Inputs that stress the tiled ball query's pruning: far-from-origin coordinates (large
    |p|^2 rounding margin), dense clusters (early exit inside the candidate scan), ragged sizes,
    hits exactly on the radius, and non-finite points and centres."""
    if case == "kitti":
        xyz = torch.rand(2, 8000, 3, generator=g) * torch.tensor([80.0, 80.0, 4.0]) - torch.tensor([40.0, 40.0, 2.0])
        return xyz, xyz[:, torch.randperm(8000, generator=g)[:3000]].contiguous(), [(0.4, 64), (1.5, 32)]
    if case == "clusters":
        c = torch.rand(2, 20, 3, generator=g) * 2 - 1
        xyz = (c[:, torch.randint(0, 20, (6000,), generator=g)] + 0.02 * torch.randn(2, 6000, 3, generator=g))
        xyz[:, ::7] = torch.rand(2, xyz[:, ::7].shape[1], 3, generator=g) * 2 - 1
        return xyz, xyz[:, :2500].contiguous(), [(0.05, 64), (0.1, 256), (0.3, 16)]
    if case == "ragged":
        xyz = torch.rand(3, 1000, 3, generator=g) * 2 - 1
        return xyz, torch.rand(3, 77, 3, generator=g) * 2 - 1, [(0.2, 128), (0.5, 8)]
    if case == "boundary":
        # dyadic grid: every d2 is exact, many exactly equal to r^2
        xyz = torch.randint(-16, 17, (2, 4096, 3), generator=g).float() / 16
        return xyz, xyz[:, :1500].contiguous(), [(0.25, 64), (0.125, 32), (0.5, 200)]
    if case == "nonfinite":
        xyz = torch.randint(-16, 17, (2, 3000, 3), generator=g).float() / 16
        ctr = xyz[:, :700].clone()
        xyz[0, 1234, 1] = float("nan")
        xyz[1, 2999, 0] = float("inf")
        ctr[0, 5, 2] = float("nan")
        ctr[1, 600, 0] = float("-inf")
        return xyz, ctr, [(0.25, 64), (0.5, 16)]
    if case == "clouds16":
        # B % 8 == 0: the tiled kernel's XCD-aware cloud mapping
        xyz = torch.randint(-16, 17, (16, 2000, 3), generator=g).float() / 16
        return xyz, xyz[:, :600].contiguous(), [(0.25, 64)]
    if case == "wide":
        # above 16384 points: the large-bitmap tiled instantiation (C5's sa1 uses N = 65536)
        xyz = torch.randint(-32, 33, (1, 20000, 3), generator=g).float() / 32
        return xyz, xyz[:, :900].contiguous(), [(0.125, 64), (0.25, 256)]
    if case == "untiled":
        # above the tiled path's 65536 points: the index-order streaming kernel
        xyz = torch.randint(-32, 33, (1, 66000, 3), generator=g).float() / 32
        return xyz, xyz[:, :600].contiguous(), [(0.125, 64)]
    raise ValueError(case)


@pytest.mark.parametrize("case", ["kitti", "clusters", "ragged", "boundary", "nonfinite", "wide", "untiled", "clouds16"])
def test_ball_query_pruned_vs_oracle(cuda, case):
    """The spatially pruned fp32 ball query (tiles + per-wave candidate bitmap) against the
    oracle (pointnet2_utils.py:87-107 restated); exact where every d2 is exact (dyadic inputs),
    else only radius-boundary rounding may differ."""
    import oracle as O
    from dvcp import ops
    g = torch.Generator().manual_seed(["kitti", "clusters", "ragged", "boundary", "nonfinite", "wide", "untiled", "clouds16"].index(case) + 140)
    xyz, ctr, radii = _bq_case(case, g)
    for r, ns in radii:
        ns = min(ns, xyz.shape[1])
        want = O.query_ball_point(r, ns, xyz, ctr)
        cnt, lst, pad = ops.ball_query(xyz.to(cuda), ctr.to(cuda), r, ns, padded=True)
        got = pad.cpu()
        if case in ("boundary", "nonfinite", "wide", "untiled", "clouds16"):
            assert torch.equal(got, want), (case, r, ns)
        else:
            assert ball_mismatch_ok(xyz, ctr, got, want, r), (case, r, ns)
        # compact form agrees with the padded one
        cnt, lst = cnt.cpu(), lst.cpu().long()
        for b in range(xyz.shape[0]):
            for s in range(0, ctr.shape[1], 53):
                c = int(cnt[b, s])
                assert torch.equal(lst[b, s, :c], got[b, s, :c])


def test_square_distance(cuda):
    import oracle as O
    import dvcp.pointnet2_utils as P
    g = torch.Generator().manual_seed(104)
    a, b = torch.rand(2, 300, 3, generator=g), torch.rand(2, 700, 3, generator=g)
    got = P.square_distance(a.to(cuda), b.to(cuda)).cpu()
    assert torch.equal(got, O.square_distance(a, b))


# ---------------------------------------------------------------------------------------- kNN
@pytest.mark.parametrize("name", ["knn_f32", "knn_dyadic"])
def test_knn_golden(cuda, name):
    from dvcp.knn import KNN
    z = golden(name)
    d, i = KNN(k=32, transpose_mode=True)(T(z["ref"], cuda), T(z["qry"], cuda))
    assert torch.equal(i.cpu(), T(z["idx"]))
    assert torch.equal(d.cpu(), T(z["dist"]))


@pytest.mark.parametrize("method", ["tiled", "tiled_insert", "brute", "grid"])
@pytest.mark.parametrize("name", ["knn_f32", "knn_dyadic"])
def test_knn_methods_golden(cuda, name, method):
    """Every kNN method on the golden fixtures (forced regardless of M)."""
    from dvcp import ops
    z = golden(name)
    d, _, i = ops.knn(T(z["ref"], cuda), T(z["qry"], cuda), 32, method=method)
    assert torch.equal(i.cpu(), T(z["idx"]))
    assert torch.equal(d.cpu(), T(z["dist"]))


def _c3_knn_inputs(cuda, M=10000, Q=20000, B=2, seed=113):
    """C3 shape: FE-like target points, candidate-grid-like queries partly far outside the cloud
    (as the R_init-only transform produces), and exact duplicates (ties)."""
    from dvcp.synthetic import rot_xyz
    g = torch.Generator().manual_seed(seed)
    ref = (torch.rand(B, M, 3, generator=g) * 2 - 1)
    ref = ref @ torch.from_numpy(rot_xyz(0.4, 1.1, 2.0)).float().T + 0.7
    if M >= 5100:
        ref[:, 5000:5100] = ref[:, 100:200]                   # duplicated points -> equal distances
    qry = torch.rand(B, Q, 3, generator=g) * 8 - 4             # many queries outside the cloud
    return ref.to(cuda), qry.to(cuda)


@pytest.mark.parametrize("method", ["tiled", "tiled_insert", "grid"])
@pytest.mark.parametrize("k", [1, 5, 20, 32])
def test_knn_method_equals_brute_full_size(cuda, k, method):
    from dvcp import ops
    ref, qry = _c3_knn_inputs(cuda)
    d1, i1, _ = ops.knn(ref, qry, k, method="brute")
    d2, i2, _ = ops.knn(ref, qry, k, method=method)
    assert torch.equal(i1, i2) and torch.equal(d1, d2)


@pytest.mark.parametrize("M,Q,k", [(16384, 3001, 32), (8193, 777, 16), (100, 1000, 32), (20, 300, 32), (1, 65, 4),
                                   (64, 64, 32), (4096, 1, 8), (5000, 900, 17), (700, 130, 31)])
def test_knn_tiled_edges_equal_brute(cuda, M, Q, k):
    """Tile-count boundaries (1, 2, 129, 256 tiles; partial last tile), fewer references than k
    (slots past M are (inf, -1) like knn.hip), a single query, ragged wave tails."""
    from dvcp import ops
    ref, qry = _c3_knn_inputs(cuda, M=M, Q=Q, B=3, seed=M + Q)
    qry[:, : Q // 3] = qry[:, :1]                              # many identical queries
    d1, i1, _ = ops.knn(ref, qry, k, method="brute")
    d2, i2, i64 = ops.knn(ref, qry, k, method="tiled")
    assert torch.equal(i1, i2) and torch.equal(d1, d2)
    assert torch.equal(i64, i2.long())


@pytest.mark.parametrize("B", [8, 16])
def test_knn_tiled_xcd_clouds_equal_brute(cuda, B):
    """B % 8 == 0 runs the tiled query kernel's XCD-aware cloud mapping (XCD x takes clouds x,
    x + 8, ...); every cloud must still get its own queries and references."""
    from dvcp import ops
    ref, qry = _c3_knn_inputs(cuda, M=4000, Q=1500, B=B, seed=B)
    d1, i1, _ = ops.knn(ref, qry, 32, method="brute")
    d2, i2, _ = ops.knn(ref, qry, 32, method="tiled")
    assert torch.equal(i1, i2) and torch.equal(d1, d2)


@pytest.mark.parametrize("k", [32, 20])
def test_knn_tiled_dyadic_ties_full(cuda, k):
    """Coordinates on a 1/8 grid: nearly every distance is tied; order must be (d2, index).  k = 20
    runs the 32-key selection kernel and keeps the first k (ties at the k-th slot included)."""
    from dvcp import ops
    g = torch.Generator().manual_seed(7)
    ref = (torch.randint(-16, 17, (2, 12000, 3), generator=g).float() / 8).to(cuda)
    qry = (torch.randint(-20, 21, (2, 5000, 3), generator=g).float() / 8).to(cuda)
    d1, i1, _ = ops.knn(ref, qry, k, method="brute")
    for method in ("tiled", "tiled_insert"):
        d2, i2, _ = ops.knn(ref, qry, k, method=method)
        assert torch.equal(i1, i2) and torch.equal(d1, d2), method


def test_knn_k1_transpose_false(cuda):
    from dvcp.knn import KNN
    z = golden("knn_k1")
    ref, qry = T(z["ref"], cuda).transpose(1, 2), T(z["qry"], cuda).transpose(1, 2)
    d, i = KNN(k=1, transpose_mode=False)(ref, qry)
    assert torch.equal(i.cpu(), T(z["idx"])) and torch.equal(d.cpu(), T(z["dist"]))


def test_knn_f64_reference_is_cast(cuda):
    import oracle as O
    from dvcp.knn import KNN
    g = torch.Generator().manual_seed(105)
    ref = torch.rand(1, 800, 3, generator=g, dtype=torch.float64)
    qry = torch.rand(1, 900, 3, generator=g, dtype=torch.float64)
    dw, iw = O.KNN(k=16, transpose_mode=True)(ref, qry)
    d, i = KNN(k=16, transpose_mode=True)(ref.to(cuda), qry.to(cuda))
    assert torch.equal(i.cpu(), iw) and torch.equal(d.cpu(), dw)


# ------------------------------------------------------------------------------- voxel grid
def test_voxelize_golden(cuda):
    import dvcp
    z = golden("voxel")
    pts = T(z["pts"], cuda)
    assert torch.equal(dvcp.voxelize(pts, 2.0, 0.4).cpu(), T(z["cand_r2"]))
    assert torch.equal(dvcp.voxelize(pts, 1.0, 0.4).cpu(), T(z["cand_r1"]))
    assert torch.equal(dvcp.voxelize_point(pts[0, 1], 2.0, 0.4).cpu(), T(z["cand_r2"])[0, 1])


# ------------------------------------------------------------------------ set abstraction
@pytest.mark.parametrize("layout,normals,B", [("channel_first", False, 2), ("channel_first", True, 2),
                                              ("point_major", False, 2), ("point_major", True, 2),
                                              ("point_major", False, 8), ("point_major", False, 16)])
def test_set_abstraction_vs_oracle(cuda, normals, layout, B):
    """All three SA tables.  Channel-first features run the row-per-thread kernel; point-major
    (each point's channels contiguous, as the forward produces them) the fp32 MFMA kernel for
    the two-layer tables.  B = 8 and 16 run the MFMA kernel's XCD-aware centre mapping (clouds
    x, x + 8, ... on XCD x)."""
    import oracle as O
    import dvcp.pointnet2_utils as P
    from tests_helpers import randomize_bn
    g = torch.Generator().manual_seed(106)
    N, S = 3000, 700
    dt = torch.float64 if normals else torch.float32
    for cfg in O.fe_config(use_normal=normals, npoint=S):
        torch.manual_seed(7)
        ref = O.PointNetSetAbstraction(**cfg).eval()
        randomize_bn(ref)
        mine = P.PointNetSetAbstraction(**cfg).eval()
        mine.load_state_dict(ref.state_dict())
        mine.to(cuda)
        xyz = (torch.rand(B, 3, N, generator=g, dtype=torch.float64) * 2 - 1).to(dt)
        D = cfg["in_channel"] - 3
        feats = torch.randn(B, D, N, generator=g, dtype=dt if D == 3 else torch.float32) if D else None
        start = torch.randint(0, N, (B,), generator=g)
        gfeats = None
        if feats is not None:
            gfeats = feats.to(cuda)
            if layout == "point_major":
                gfeats = gfeats.transpose(1, 2).contiguous().transpose(1, 2)  # (B, D, N) view, fd = 1
        with torch.no_grad():
            O_xyz, O_f = _sa_oracle(ref, xyz, feats, start)
            G_xyz, G_f = mine(xyz.to(cuda), gfeats, start=start)
        assert torch.equal(G_xyz.cpu(), O_xyz)
        torch.testing.assert_close(G_f.cpu(), O_f, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("table", [0, 1, 2])
def test_sa_split3_accuracy(cuda, table):
    """The MFMA tables run their bf16 layers as a three-way bf16 split on the matrix cores
    (csrc/sa_mlp_mfma.hip: layer 2 of sa2 / sa3, layers 2 and 3 of sa1).  On the same groups (the
    GPU ball query's lists) the error against an fp64 evaluation of pointnet2_utils.py:195-200 must
    be of the size of an fp32 evaluation's error (torch fp32 on the CPU, the reference's own
    arithmetic), and within the fp32 tolerance of it.  sa1 (nsample 256) at ~3/4 of nsample hits per
    ball runs up to 16 half tiles per centre."""
    import copy
    import oracle as O
    import dvcp.pointnet2_utils as P
    from dvcp import ops
    from tests_helpers import randomize_bn
    g = torch.Generator().manual_seed(211 + table)
    cfg = O.fe_config(use_normal=False, npoint=2000)[table]
    B, N, S, ns, r = 2, 6000, 2000, cfg["nsample"], cfg["radius"]
    D = cfg["in_channel"] - 3
    torch.manual_seed(11)
    mine = P.PointNetSetAbstraction(**cfg).eval()
    randomize_bn(mine)
    side = r * (4.19 * N / (0.75 * ns)) ** (1.0 / 3.0)  # ~3/4 of nsample hits per ball
    xyz = ((torch.rand(B, 3, N, generator=g, dtype=torch.float64) - 0.5) * side).float()
    feats = torch.randn(B, N, D, generator=g)           # point-major rows, as the forward stores them
    gx, gf = xyz.to(cuda), feats.to(cuda)
    ctr = gx[:, :, :S].contiguous()
    mine_g = copy.deepcopy(mine).to(cuda)
    count, lst, _ = ops.ball_query(gx, ctr, r, ns, pdim=2, cdim_pts=2)
    out = ops.sa_group_mlp(gx, ctr, gf.transpose(1, 2) if D else None, count, lst, ns, mine_g.chans,
                           mine_g.packed_params(), xyz_pdim=2, feat_ddim=1, feat_pdim=2).cpu()  # (B, S, C_last)
    cnt = count.cpu().long().clamp(1, ns)
    idx = lst.cpu().long()
    idx = torch.where(torch.arange(ns).view(1, 1, ns) < cnt.unsqueeze(-1), idx, idx[:, :, :1])  # :104 padding
    bi = torch.arange(B).view(B, 1, 1)
    gxyz = xyz.transpose(1, 2)[bi, idx] - xyz.transpose(1, 2)[:, :S].unsqueeze(2)  # fp32 differences
    rows = (torch.cat([gxyz, feats[bi, idx]], dim=-1) if D else gxyz).permute(0, 3, 2, 1)  # (B, C0, ns, S)

    def mlp(m, x):
        for conv, bn in zip(m.mlp_convs, m.mlp_bns):
            x = torch.relu(bn(conv(x)))
        return torch.max(x, 2)[0].transpose(1, 2)
    with torch.no_grad():
        ref64 = mlp(copy.deepcopy(mine).double(), rows.double())
        ref32 = mlp(mine, rows)
    err_gpu = float((out.double() - ref64).abs().max())
    err_f32 = float((ref32.double() - ref64).abs().max())
    scale = float(ref64.abs().max())
    print(f"sa table {table}: max |gpu - fp64| {err_gpu:.3e}, max |fp32 cpu - fp64| {err_f32:.3e}, |ref| {scale:.3f}")
    assert err_gpu <= 4.0 * err_f32 + 1e-7 * scale
    torch.testing.assert_close(out, ref32, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("table", [0, 1, 2])
def test_sa_empty_ball_gives_zero(cuda, table):
    """A centre whose ball holds no point (count 0; the reference would gather index N, :104) gets a
    zero row from every table, and its list row is never read (filled here with an out-of-range
    index); the other centres are unchanged.  20000 centres: above 16384 the MFMA kernels give a
    wave several centres, so an empty centre sits between centres with hits in one wave."""
    import dvcp.pointnet2_utils as P
    import oracle as O
    from dvcp import ops
    from tests_helpers import randomize_bn
    g = torch.Generator().manual_seed(231 + table)
    cfg = O.fe_config(use_normal=False, npoint=5000)[table]
    B, N, S, ns, r = 4, 5000, 5000, cfg["nsample"], cfg["radius"]
    D = cfg["in_channel"] - 3
    torch.manual_seed(13)
    mine = P.PointNetSetAbstraction(**cfg).eval()
    randomize_bn(mine)
    mine = mine.to(cuda)
    gx = ((torch.rand(B, 3, N, generator=g, dtype=torch.float64) - 0.5) * 4).float().to(cuda)
    gf = torch.randn(B, N, D, generator=g).to(cuda) if D else None
    ctr = gx[:, :, :S].contiguous()
    count, lst, _ = ops.ball_query(gx, ctr, r, ns, pdim=2, cdim_pts=2)
    args = dict(xyz_pdim=2, feat_ddim=1, feat_pdim=2)
    feat = gf.transpose(1, 2) if D else None
    full = ops.sa_group_mlp(gx, ctr, feat, count, lst, ns, mine.chans, mine.packed_params(), **args)
    empty = torch.zeros(B, S, dtype=torch.bool, device=cuda)
    empty[:, ::7] = True
    count2 = torch.where(empty, torch.zeros_like(count), count)
    lst2 = torch.where(empty.unsqueeze(-1), torch.full_like(lst, 1 << 30), lst)
    got = ops.sa_group_mlp(gx, ctr, feat, count2, lst2, ns, mine.chans, mine.packed_params(), **args)
    torch.cuda.synchronize()
    assert torch.equal(got[empty], torch.zeros_like(got[empty]))
    assert torch.equal(got[~empty], full[~empty])


def _sa_oracle(ref, xyz, feats, start):
    import oracle as O
    orig = O.ref_r.farthest_point_sample

    def fps_fixed(x, npoint, start=None, _fixed=start):
        return orig(x, npoint, _fixed)

    O.ref_r.farthest_point_sample = fps_fixed
    try:
        return ref(xyz, feats)
    finally:
        O.ref_r.farthest_point_sample = orig


# ------------------------------------------------------------------------------ heads, top-k
def test_fe_head_and_weighting(cuda):
    import oracle as O
    import dvcp
    g = torch.Generator().manual_seed(107)
    torch.manual_seed(3)
    fe = O.feat_extraction_layer(use_normal=False, npoint=16)
    wl = O.weighting_layer()
    x = torch.randn(5000, 64, generator=g)
    mine_fe = dvcp.feat_extraction_layer(use_normal=False, npoint=16).eval()
    mine_fe.load_state_dict(fe.state_dict())
    mine_wl = dvcp.weighting_layer().eval()
    mine_wl.load_state_dict(wl.state_dict())
    mine_fe.to(cuda), mine_wl.to(cuda)
    from dvcp import ops
    feat, score = ops.fe_head(x.to(cuda), mine_fe.fc_params(mine_wl), with_score=True)
    with torch.no_grad():
        f_ref = fe.fc(x)
        s_ref = wl.fc3(wl.fc2(wl.fc1(f_ref)))[:, 0]
    torch.testing.assert_close(feat.cpu(), f_ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(score.cpu(), s_ref, rtol=1e-5, atol=1e-6)
    s2 = mine_wl.scores(f_ref.view(1, 5000, 32).to(cuda))
    torch.testing.assert_close(s2.cpu()[0], s_ref, rtol=1e-5, atol=1e-6)


def test_row_map_entries_equal_gather(cuda):
    """dvcp_sa_group_mlp_rows_ws and dvcp_fe_head_rows (the FE's folded FPS-order gathers) give
    bit-for-bit what the plain entries give on the torch-gathered tables, including repeated and
    out-of-order rows."""
    import dvcp
    import dvcp.pointnet2_utils as P
    from dvcp import ops
    g = torch.Generator().manual_seed(121)
    B, Nf, N = 3, 1200, 1000
    for D, chans, radius in ((32, (35, 32, 64), 0.2), (64, (67, 64, 64), 0.4)):
        sa = P.PointNetSetAbstraction(npoint=N, radius=radius, nsample=64, in_channel=3 + D, mlp=list(chans[1:]))
        sa = sa.eval().to(cuda)
        table = torch.randn(B, Nf, D, generator=g).to(cuda)
        rows = torch.randint(0, Nf, (B, N), generator=g).to(cuda)
        xyz = (torch.rand(B, 3, N, generator=g) * 2 - 1).to(cuda)
        count, lst, _ = ops.ball_query(xyz, xyz, radius, 64, pdim=2, cdim_pts=2)
        gathered = torch.gather(table, 1, rows.unsqueeze(-1).expand(-1, -1, D))          # (B, N, D)
        want = ops.sa_group_mlp(xyz, xyz, gathered.permute(0, 2, 1), count, lst, 64, chans, sa.packed_params(),
                                xyz_pdim=2, feat_ddim=1, feat_pdim=2)
        got = ops.sa_group_mlp_rows(xyz, xyz, table, rows, count, lst, 64, chans, sa.packed_params())
        assert torch.equal(got, want), D
    fe = dvcp.feat_extraction_layer(use_normal=False, npoint=16).eval().to(cuda)
    wl = dvcp.weighting_layer().eval().to(cuda)
    x = torch.randn(B, Nf, 64, generator=g).to(cuda)
    rows = torch.randint(0, Nf, (B, N), generator=g).to(cuda)
    gathered = torch.gather(x, 1, rows.unsqueeze(-1).expand(-1, -1, 64)).reshape(B * N, 64)
    f1, s1 = ops.fe_head(gathered, fe.fc_params(wl), with_score=True)
    f2, s2 = ops.fe_head_rows(x, rows, fe.fc_params(wl), with_score=True)
    assert torch.equal(f1, f2) and torch.equal(s1, s2)


def test_topk(cuda):
    from dvcp import ops
    g = torch.Generator().manual_seed(108)
    s = torch.rand(3, 10000, generator=g)
    got = ops.topk(s.to(cuda), 64).cpu()
    assert torch.equal(got, torch.topk(s, 64, dim=1).indices)
    tied = torch.tensor([[1.0, 5.0, 5.0, 2.0, 5.0, 0.0]])
    assert ops.topk(tied.to(cuda), 4).cpu().tolist() == [[1, 2, 4, 3]]  # value desc, index asc


@pytest.mark.parametrize("case", ["all_equal", "few_values", "negative", "k_eq_s", "k1", "ragged", "k256",
                                  "neg_inf_ragged"])
def test_topk_radix_select_cases(cuda, case):
    """The radix-select top-k (head_topk.hip) against value-descending, index-ascending order:
    massive ties (the select runs into the index bits), mixed signs, K = S, K = 1, S not a
    multiple of the workgroup, C5's K = 256."""
    import numpy as np
    from dvcp import ops
    g = torch.Generator().manual_seed(118)
    B, S, K = 3, 10000, 64
    if case == "all_equal":
        s = torch.full((B, S), 0.75)
    elif case == "few_values":
        s = torch.randint(0, 5, (B, S), generator=g).float() * 0.25
    elif case == "negative":
        s = torch.randn(B, S, generator=g)
    elif case == "k_eq_s":
        S = K = 700
        s = torch.rand(B, S, generator=g)
    elif case == "k1":
        K = 1
        s = torch.rand(B, S, generator=g)
    elif case == "ragged":
        S, K = 3333, 50
        s = torch.randint(0, 40, (B, S), generator=g).float()
    elif case == "neg_inf_ragged":
        # K = S, S not a multiple of 1024, scores of both signs and -inf: the K-th key's top byte
        # is the padding slots' (0), which must still never be selected
        S = K = 1500
        s = torch.randn(B, S, generator=g)
        s[:, ::3] = -float("inf")
        s[1, 5:9] = -3.0e38
    else:
        S, K = 16384, 256
        s = torch.rand(B, S, generator=g)
    got = ops.topk(s.to(cuda), K).cpu().numpy()
    for b in range(B):
        v = s[b].numpy()
        want = np.lexsort((np.arange(S), -v))[:K]  # value descending, then index ascending
        assert np.array_equal(got[b], want), case


# ------------------------------------------------------------------------------ DFE / CPG
def test_dfe_vs_oracle(cuda):
    import oracle as O
    import dvcp
    g = torch.Generator().manual_seed(109)
    torch.manual_seed(4)
    ref = O.feat_embedding_layer()
    mine = dvcp.feat_embedding_layer().eval()
    mine.load_state_dict(ref.state_dict())
    mine.to(cuda)
    Xs = torch.randn(2, 64, 32, 35, generator=g, dtype=torch.float64)
    Xt = torch.randn(2, 5, 27, 32, 35, generator=g)
    with torch.no_grad():
        torch.testing.assert_close(mine(Xs.to(cuda), src=True).cpu(), ref(Xs, src=True), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(mine(Xt.to(cuda), src=False).cpu(), ref(Xt, src=False), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("literal", [False, True], ids=["collapsed", "literal"])
@pytest.mark.parametrize("f64", [False, True])
def test_dfe_tgt_fused_vs_oracle(cuda, f64, literal):
    """The fused target DFE against the oracle's materialised Get_Cat_Feat_Tgt + feat_embedding_layer:
    the default kernel collapses fc3 fc2 fc1 into one map (SURVEY App. A.3 Q14 deviation, formed in
    fp64 and rounded once), dvcp_dfe_tgt_literal chains the three layers as written; both within
    1e-5, the same bar."""
    import oracle as O
    import dvcp
    from dvcp import ops
    g = torch.Generator().manual_seed(110)
    dt = torch.float64 if f64 else torch.float32
    B, K, G, M = 2, 3, 6, 900
    C = G ** 3
    torch.manual_seed(5)
    dfe_ref = O.feat_embedding_layer()
    mine = dvcp.feat_embedding_layer().eval()
    mine.load_state_dict(dfe_ref.state_dict())
    mine.to(cuda)
    ref_xyz = (torch.rand(B, M, 3, generator=g, dtype=torch.float64) * 2 - 1).to(dt)
    ref_feat = torch.randn(B, M, 32, generator=g)
    cand = O.voxelize(torch.rand(B, K, 3, generator=g, dtype=torch.float64) - 0.5, 1.0, 0.4)
    with torch.no_grad():
        cat = O.Get_Cat_Feat_Tgt()(cand, torch.zeros(B, K, 3), ref_xyz, ref_feat)
        want = dfe_ref(cat, src=False)
    qry = cand.view(B, K * C, 3).to(cuda)
    dist, idx, _ = ops.knn(ref_xyz.to(cuda), qry, 32, ref_pdim=1, qry_pdim=1)
    got = ops.dfe_tgt(ref_xyz.to(cuda), ref_feat.to(cuda), qry, dist, idx, mine.packed_params(), ref_pdim=1,
                      literal=literal)
    print(f"dfe_tgt literal={literal} f64={f64}: max|err| {float((got.view(B, K, C, 32).cpu() - want).abs().max()):.2e}")
    torch.testing.assert_close(got.view(B, K, C, 32).cpu(), want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("r", [1.0, 2.0])
def test_cpg_vs_oracle(cuda, r):
    import oracle as O
    import dvcp
    g = torch.Generator().manual_seed(111)
    torch.manual_seed(6)
    ref = O.cpg()
    mine = dvcp.cpg().eval()
    mine.load_state_dict(ref.state_dict())
    mine.to(cuda)
    G = int(2 * r / 0.4 + 1)
    C = G ** 3
    B, K = 2, 8
    src = torch.randn(B, K, 1, 32, generator=g)
    tgt = torch.randn(B, K, C, 32, generator=g).permute(0, 1, 3, 2)   # the reference's permuted view
    cand = torch.randn(B, K, C, 3, generator=g)
    with torch.no_grad(), O.tracing() as tr:
        want = ref(src, tgt, cand, r, 0.4)
    got, w = mine(src.to(cuda), tgt.to(cuda), cand.to(cuda), r, 0.4, return_weights=True)
    torch.testing.assert_close(got.cpu(), want, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(w.cpu(), dict(tr)["cpg_weight"], rtol=1e-4, atol=1e-7)


# ------------------------------------------------------------------------------ pose solve
def test_rigid_golden(cuda):
    import dvcp
    z = golden("rigid")
    x, y = T(z["x"], cuda), T(z["y"], cuda)
    Rt, tt = T(z["R_true"], cuda), T(z["t_true"], cuda)
    loss, R, t = dvcp.deepVCP_loss(x, y, Rt, tt, 0.5)
    torch.testing.assert_close(R.cpu(), T(z["R"]), rtol=0, atol=1e-9)
    torch.testing.assert_close(t.cpu(), T(z["t"]), rtol=0, atol=1e-9)
    torch.testing.assert_close(loss.cpu(), T(z["loss"]), rtol=1e-9, atol=1e-12)
    R1, t1 = dvcp.get_rigid_transform(x.transpose(1, 2), y.double().transpose(1, 2))
    torch.testing.assert_close(R1.cpu(), T(z["R1"]), rtol=0, atol=1e-9)
    torch.testing.assert_close(t1.cpu(), T(z["t1"]), rtol=0, atol=1e-9)


def test_rigid_exact_rotation_and_reflection(cuda):
    import dvcp
    from dvcp.synthetic import rot_xyz
    g = torch.Generator().manual_seed(112)
    x = torch.randn(2, 3, 50, generator=g, dtype=torch.float64)
    R = torch.from_numpy(np.stack([rot_xyz(0.3, 1.2, -2.0), np.diag([1.0, 1.0, -1.0])]))
    t = torch.tensor([[[0.5], [-1.0], [2.0]], [[0.0], [0.0], [0.0]]], dtype=torch.float64)
    Rg, tg = dvcp.get_rigid_transform(x.to(cuda), (R @ x + t).to(cuda))
    torch.testing.assert_close(Rg.cpu(), R, rtol=0, atol=1e-12)     # Q13: the reflection is returned as-is
    torch.testing.assert_close(tg.cpu(), t, rtol=0, atol=1e-12)


# ----------------------------------------------------------------- registration error (harness)
def test_registration_error_vs_oracle(cuda):
    """dvcp_registration_error against scipy's Euler angles (train.py:112-120, C8 fixed)."""
    import oracle as O
    from scipy.spatial.transform import Rotation
    from dvcp import ops
    g = torch.Generator().manual_seed(120)
    B = 256
    Rp = torch.tensor(Rotation.random(B, random_state=1).as_matrix())
    Rg = torch.tensor(Rotation.random(B, random_state=2).as_matrix())
    Rp[:64] = Rg[:64] @ torch.tensor(Rotation.from_rotvec(1e-3 * torch.randn(64, 3, generator=g,
                                                                               dtype=torch.float64).numpy()).as_matrix())
    Rp[7] = torch.diag(torch.tensor([1.0, -1.0, 1.0], dtype=torch.float64))  # reflection: NaN like scipy
    tp = torch.randn(B, 3, 1, generator=g, dtype=torch.float64)
    tg = torch.randn(B, 3, 1, generator=g, dtype=torch.float64)
    want_r, want_t = O.registration_errors(Rp, tp, Rg, tg)
    got_r, got_t = ops.registration_error(Rp.to(cuda), tp.to(cuda), Rg.to(cuda), tg.to(cuda))
    torch.testing.assert_close(got_r.cpu(), want_r, rtol=0, atol=1e-9, equal_nan=True)
    torch.testing.assert_close(got_t.cpu(), want_t, rtol=0, atol=1e-12)
    # one ground-truth pose broadcast over the batch
    got_r1, _ = ops.registration_error(Rp.to(cuda), tp.to(cuda), Rg[:1].to(cuda), tg[:1].to(cuda))
    want_r1, _ = O.registration_errors(Rp, tp, Rg[:1], tg[:1])
    torch.testing.assert_close(got_r1.cpu(), want_r1, rtol=0, atol=1e-9, equal_nan=True)


def test_sa_mlp_plain_entry_matches_workspace_entry(cuda):
    """dvcp_sa_group_mlp (no workspace: layer 1 per row, BN after the GEMM) and
    dvcp_sa_group_mlp_ws (per-point U, BN folded, Hilbert visiting order) agree to fp32 rounding
    on the sa3 table (67-64-64) with per-point centres, as the forward runs it."""
    import dvcp.pointnet2_utils as P
    from dvcp import _lib, ops
    from tests_helpers import randomize_bn
    g = torch.Generator().manual_seed(121)
    B, N = 2, 3000
    torch.manual_seed(8)
    sa = P.PointNetSetAbstraction(npoint=N, radius=0.4, nsample=64, in_channel=67, mlp=[64, 64]).eval()
    randomize_bn(sa)
    sa.to(cuda)
    xyz = (torch.rand(B, 3, N, generator=g) * 2 - 1).to(cuda)
    feat = torch.randn(B, N, 64, generator=g).to(cuda).transpose(1, 2)  # (B, 64, N), point-major memory
    count, lst, _ = ops.ball_query(xyz, xyz, 0.4, 64, pdim=2, cdim_pts=2)
    got_ws = ops.sa_group_mlp(xyz, xyz, feat, count, lst, 64, sa.chans, sa.packed_params(), xyz_pdim=2,
                              feat_ddim=1, feat_pdim=2)
    ch = torch.tensor(list(sa.chans), dtype=torch.int32)
    plain = torch.empty_like(got_ws)
    st = feat.stride()
    _lib.call("dvcp_sa_group_mlp", _lib.F32, _lib.ptr(xyz), xyz.stride(0), xyz.stride(1), xyz.stride(2), N,
              _lib.ptr(xyz), xyz.stride(0), xyz.stride(1), xyz.stride(2), N, B, _lib.F32, _lib.ptr(feat), st[0],
              st[1], st[2], 64, _lib.ptr(count), _lib.ptr(lst), 64, 2, _lib.ctypes.c_void_p(ch.data_ptr()),
              _lib.ptr(sa.packed_params()), _lib.ptr(plain), _lib.stream())
    torch.testing.assert_close(got_ws, plain, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("fix", [True, False])
def test_paper_pose_vs_checker(cuda, fix):
    """dvcp.paper (DeepVCP paper Sec. 3.4-3.5): weighted, reflection-corrected
    Kabsch and the paper's two-term loss against the numpy restatement (oracle/paper.py) within
    1e-9, on noisy correspondences with random weights and on mirrored sets (reflections)."""
    import numpy as np
    from oracle import paper as OP
    import dvcp
    g = np.random.default_rng(31)
    B, n = 6, 64
    x = g.standard_normal((B, 3, n))
    R_true = np.stack([np.linalg.qr(g.standard_normal((3, 3)))[0] for _ in range(B)])
    R_true *= np.sign(np.linalg.det(R_true))[:, None, None]
    t_true = g.standard_normal((B, 3))
    y = R_true @ x + t_true[..., None] + 0.05 * g.standard_normal((B, 3, n))
    y[3] = np.diag([1.0, 1.0, -1.0]) @ x[3]           # mirrored pairs: the fix decides
    y[4] = np.diag([-1.0, 1.0, 1.0]) @ x[4] + 0.3
    w = g.random((B, n)) + 0.05
    w[5, :10] = 0.0
    loss_o, R_o, t_o = OP.deepvcp_loss_paper(x, y, w, R_true, t_true, 0.5, reflection_fix=fix)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)
    loss, R, t = dvcp.paper.deepVCP_loss_paper(T(x.transpose(0, 2, 1)), T(y.transpose(0, 2, 1)), T(w), T(R_true),
                                               T(t_true[..., None]), 0.5, reflection_fix=fix)
    assert np.allclose(R.cpu().numpy(), R_o, atol=1e-9)
    assert np.allclose(t.cpu().numpy()[..., 0], t_o, atol=1e-9)
    assert abs(float(loss) - loss_o) <= 1e-9 * max(1.0, abs(loss_o))
    dets = np.linalg.det(R.cpu().numpy())
    assert (np.abs(dets - 1.0) < 1e-9).all() if fix else (dets[3] < 0 and dets[4] < 0)
    R2, t2 = dvcp.paper.weighted_rigid_transform(T(x), T(y), T(w), reflection_fix=fix)
    assert torch.equal(R2, R) and torch.equal(t2, t)


def test_dfe_tgt_packed_point_rows_bit_identical(cuda):
    """ops.dfe_tgt hands fp32 points to the kernel as (x, y, z, 0) rows (dvcp_points_pack4, one
    16-byte gather per neighbour); the kernel on the strided (B, 3, M) layout gives the same bits.
    The pack itself copies the coordinates exactly (pad 0).  Both XCD mappings (B = 2 and 8)."""
    import dvcp
    from dvcp import _lib, ops
    from dvcp.ops import ptr, stream
    g = torch.Generator().manual_seed(113)
    mine = dvcp.feat_embedding_layer().eval().to(cuda)
    for B, Q, M in ((2, 700, 900), (8, 3000, 2000)):
        xyz = (torch.rand(B, 3, M, generator=g) * 2 - 1).to(cuda)          # (B, 3, M): the FE's layout
        feat = torch.randn(B, M, 32, generator=g).to(cuda)
        qry = (torch.rand(B, Q, 3, generator=g) * 2 - 1).to(cuda)
        dist, idx, _ = ops.knn(xyz, qry, 32, ref_pdim=2, qry_pdim=1)
        pk = ops.points_pack4(xyz, 2)
        assert torch.equal(pk[..., :3], xyz.permute(0, 2, 1)) and torch.equal(pk[..., 3], torch.zeros_like(pk[..., 3]))
        got = ops.dfe_tgt(xyz, feat, qry, dist, idx, mine.packed_params(), ref_pdim=2)
        raw = torch.empty_like(got)
        _lib.call("dvcp_dfe_tgt", _lib.F32, ptr(xyz), xyz.stride(0), xyz.stride(1), xyz.stride(2), M, ptr(feat),
                  ptr(qry), ptr(dist), ptr(idx), B, Q, ptr(mine.packed_params()), ptr(raw), stream())
        assert torch.equal(got, raw)


@pytest.mark.parametrize("f64", [False, True])
def test_dfe_tgt_fp16_features(cuda, f64):
    """BASELINE C5's fp16 feature storage (dvcp_dfe_tgt_f16): the gathered rows are widened to fp32
    and the rest is the fp32 kernel's arithmetic, so the output equals dvcp_dfe_tgt on the fp32
    table holding the same fp16-rounded values bit for bit (that kernel is checked against the
    oracle in test_dfe_tgt_fused_vs_oracle); against the unrounded table it differs by the
    features' fp16 rounding only (<= 2e-3 relative here).  Both XCD mappings (B = 2 and 8)."""
    import dvcp
    from dvcp import ops
    g = torch.Generator().manual_seed(111)
    dt = torch.float64 if f64 else torch.float32
    mine = dvcp.feat_embedding_layer().eval().to(cuda)
    for B, K, G, M in ((2, 3, 6, 900), (8, 8, 11, 2000)):
        C = G ** 3
        ref_xyz = (torch.rand(B, M, 3, generator=g, dtype=torch.float64) * 2 - 1).to(dt).to(cuda)
        feat = torch.randn(B, M, 32, generator=g).to(cuda)
        qry = ((torch.rand(B, K * C, 3, generator=g, dtype=torch.float64) * 2 - 1).float()).to(cuda)
        dist, idx, _ = ops.knn(ref_xyz, qry, 32, ref_pdim=1, qry_pdim=1)
        half = feat.half()
        got = ops.dfe_tgt(ref_xyz, half, qry, dist, idx, mine.packed_params(), ref_pdim=1)
        same = ops.dfe_tgt(ref_xyz, half.float(), qry, dist, idx, mine.packed_params(), ref_pdim=1)
        assert torch.equal(got, same)
        full = ops.dfe_tgt(ref_xyz, feat, qry, dist, idx, mine.packed_params(), ref_pdim=1)
        rel = float((got - full).abs().max() / full.abs().max())
        print(f"B={B}: fp16-feature DFE vs fp32 features: max rel {rel:.2e}")
        assert rel < 2e-3
    with pytest.raises(ValueError):
        ops.dfe_tgt(ref_xyz, half, qry, dist, idx, mine.packed_params(), ref_pdim=1, literal=True)



def test_fe_chain_with_fps_pair_equals_serial(cuda, monkeypatch):
    """The feature extractor with the opt-in paired layer-2/3 FPS (DVCP_FPS_PAIR=1) against the
    default serial chain: same centres, features and scores, bit for bit."""
    from dvcp.deep_feat_extraction import feat_extraction_layer
    g = torch.Generator().manual_seed(430)
    torch.manual_seed(430)
    fe = feat_extraction_layer(use_normal=False, npoint=4096).to(cuda).eval()
    pts = (torch.rand(2, 3, 6000, generator=g) * 2 - 1).to(cuda)
    starts = [torch.randint(0, n, (2,), generator=g) for n in (6000, 4096, 4096)]
    outs = {}
    with torch.no_grad():
        for mode in ("0", "1"):
            monkeypatch.setenv("DVCP_FPS_PAIR", mode)
            xyz, feat, _ = fe.run(pts, starts)
            torch.cuda.synchronize()
            outs[mode] = (xyz.clone(), feat.clone())
    assert torch.equal(outs["0"][0], outs["1"][0])
    assert torch.equal(outs["0"][1], outs["1"][1])
