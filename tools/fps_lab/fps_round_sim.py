"""CPU model of fps_select_kernel's round logic (csrc/fps.hip: the floor f, the 256-bin histogram
over (f, vmax], the list capacity, the candidate selection and the prefix acceptance), in fp32 like
the kernel, to count rounds, scans and rescans per reason under other parameters without a GPU.
The accepted centres are the exact FPS order (sim(...)["order"]), so a model run is also an FPS.
Study tool only (the kernel's own counters: fps_lab --stats)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "deepvcp-pointcloud-registration_amd"))


def bitlen(x):
    return int(x).bit_length()


def d2(P, c):
    d = P - c
    return ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)


def sim(P, npoint, cap=1024, target=64, smax=128, smin=16, accept=64, decay=0.9, lowmark=256):
    P = P.astype(np.float32)
    N = len(P)
    dmin = np.full(N, np.float32(1e10))
    dmin = np.minimum(d2(P, P[0]), dmin)
    vmax = np.float32(dmin.max())
    f = np.float32(0.0)
    step = 1
    rounds = scans = 0
    why = [0, 0, 0, 0]
    fb = 0
    ks = []
    order_out = [0]
    idx = np.arange(N)
    while step < npoint:
        rounds += 1
        raised = False
        scan = 0
        while True:
            scans += 1
            kf = int(np.float32(f).view(np.uint32))
            kv = max(int(np.float32(vmax).view(np.uint32)), kf + 1)
            rng = kv - kf
            shift = 0 if rng < 256 else bitlen(rng) - 8
            hit = dmin > f
            na = int(hit.sum())
            nh = ~hit
            Tf = np.float32(dmin[nh].max()) if nh.any() else np.float32(0)
            hv = dmin[hit]
            hb = np.minimum((hv.view(np.uint32).astype(np.int64) - kf) >> shift, 255)
            hist = np.bincount(hb, minlength=256)
            suf = np.cumsum(hist[::-1])[::-1]

            def lbal(need):
                k = np.nonzero(suf >= need)[0]
                return int(k.max()) if len(k) else -1

            def edge_below(b):
                return np.uint32(kf + (b << shift) - 1).view(np.float32)

            mode = 0
            bsel = 0
            if scan >= 8:
                mode = 2
            elif na == 0:
                if Tf > 0:
                    f = np.float32(np.uint32(np.float32(Tf).view(np.uint32) - 1).view(np.float32))
                    mode = 1
                    why[0] += 1
                else:
                    mode = 2
            else:
                top = lbal(1)

                def tighten():
                    return vmax if top >= 255 else min(vmax, np.uint32(kf + ((top + 1) << shift)).view(np.float32))
                if na > cap:
                    bb = max(0, lbal(4 * target))
                    while bb + 1 < 256 and suf[bb] > cap and suf[bb + 1] > 0:
                        bb += 1
                    if shift == 0 and suf[bb] > cap:
                        mode = 2
                    else:
                        if bb > 0:
                            f = edge_below(bb)
                        vmax = tighten()
                        mode = 1
                        raised = True
                        why[1] += 1
                elif na < smin and Tf > 0 and not raised:
                    f = min(np.float32(f * np.float32(0.5)),
                            np.uint32(np.float32(Tf).view(np.uint32) - 1).view(np.float32))
                    mode = 1
                    why[2] += 1
                else:
                    bsel = max(0, lbal(min(target, na)))
                    while bsel + 1 < 256 and suf[bsel] > smax and suf[bsel + 1] > 0:
                        bsel += 1
                    if suf[bsel] > smax:
                        if shift == 0:
                            mode = 2
                        else:
                            if bsel > 0:
                                f = edge_below(bsel)
                            vmax = tighten()
                            mode = 1
                            raised = True
                            why[3] += 1
            if mode == 1:
                scan += 1
                continue
            if mode == 2:
                fb += 1
                gm = dmin.max()
                j = int(np.nonzero(dmin == gm)[0].min())
                dmin = np.minimum(dmin, d2(P, P[j]))
                order_out.append(j)
                vmax = np.float32(gm)
                step += 1
                ks.append(1)
                break
            # list: hits in order (the kernel's list order differs; the capacity matters only when na > cap)
            hid = idx[hit]
            inb = hb >= bsel
            cand = hid[inb]
            cv = hv[inb]
            T = max(Tf, np.float32(hv[~inb].max()) if (~inb).any() else np.float32(0))
            if na < lowmark:
                f = np.float32(f * np.float32(decay))
            order = np.lexsort((cand, -cv.astype(np.float64)))
            cand, cv = cand[order], cv[order]
            left = npoint - step
            k = 0
            for r in range(len(cand)):
                if r >= left:
                    break
                if r > 0:
                    if not (cv[r] > T):
                        break
                    dd = d2(P[cand[:r]], P[cand[r]])
                    if (dd < cv[r]).any():
                        break
                k += 1
            k = min(k, len(cand), accept)
            for j in cand[:k]:
                dmin = np.minimum(dmin, d2(P, P[j]))
                order_out.append(int(j))
            vm = T
            if k < len(cand):
                vm = max(vm, cv[k:].max())
            vmax = np.float32(vm)
            step += k
            ks.append(k)
            break
    return dict(rounds=rounds, scans=scans, why=why, fallbacks=fb, per_round=np.mean(ks), order=order_out)


if __name__ == "__main__":
    from dvcp.synthetic import make_pairs
    src, tgt, _, _ = make_pairs(2, 16384, seed=1234)
    P = src[0].numpy().T
    import time
    for kw in [dict(decay=0.85), dict(decay=0.85, cap=2048), dict(decay=0.9), dict(decay=0.9, lowmark=128)]:
        t = time.time()
        r = sim(P, 10000, **kw)
        r.pop("order")
        print(kw, r, f"{time.time() - t:.1f}s", flush=True)
