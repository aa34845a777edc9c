"""Exact batched FPS -- numpy prototype of the GPU algorithm (diagnostics).

Checks that the batched walk reproduces the serial FPS index sequence bit for bit (fp32, the
reference's rounding: d = ((dx*dx + dy*dy) + dz*dz), strict '<' update, first-index argmax) and
reports the batch sizes.  Layout mirrors the kernel plan: points Morton-sorted, group = 64
consecutive sorted points; each group publishes its best (value desc, index asc) and the second
largest value as a bound; the walker lists each lane's best of 4 groups and bounds the rest by the
largest unlisted candidate value.

    python tools/fps_lab/batched_fps_proto.py [N npoint]
"""
import sys

import numpy as np

f32 = np.float32


def d2(px, py, pz, cx, cy, cz):
    dx, dy, dz = px - cx, py - cy, pz - cz
    return (dx * dx + dy * dy) + dz * dz


def serial_fps(x, npoint, start):
    N = len(x)
    dmin = np.full(N, f32(1e10), f32)
    out = np.empty(npoint, np.int64)
    cur = start
    for s in range(npoint):
        out[s] = cur
        d = d2(x[:, 0], x[:, 1], x[:, 2], x[cur, 0], x[cur, 1], x[cur, 2])
        dmin = np.where(d < dmin, d, dmin)
        cur = int(np.argmax(dmin))  # first index of the maximum
    return out


def morton_order(x):
    lo, hi = x.min(0), x.max(0)
    q = np.clip(((x - lo) * (16 / np.maximum(hi - lo, 1e-30))).astype(int), 0, 15)

    def spread(v):
        return (v & 1) | ((v & 2) << 2) | ((v & 4) << 4) | ((v & 8) << 6)

    cell = spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)
    return np.argsort(cell, kind="stable")


def maxd2(blo, bhi, c):
    """Rounding-safe upper bound of d2(p, c) over a box: per axis the larger |face - c|."""
    ex = np.maximum(np.abs(blo[:, 0] - c[0]), np.abs(bhi[:, 0] - c[0]))
    ey = np.maximum(np.abs(blo[:, 1] - c[1]), np.abs(bhi[:, 1] - c[1]))
    ez = np.maximum(np.abs(blo[:, 2] - c[2]), np.abs(bhi[:, 2] - c[2]))
    return (ex * ex + ey * ey) + ez * ez


def batched_fps(x, npoint, start, S=64, lanes=64):
    N = len(x)
    order = morton_order(x)
    G = -(-N // S)
    pad = G * S - N
    pid = np.concatenate([order, np.full(pad, -1)])
    xs = np.concatenate([x[order], np.zeros((pad, 3), f32)]).astype(f32)
    real = pid >= 0
    dmin = np.where(real, f32(1e10), f32(-1)).astype(f32)
    gl = np.where(real[:, None], xs, np.inf).reshape(G, S, 3).min(1).astype(f32)
    gh = np.where(real[:, None], xs, -np.inf).reshape(G, S, 3).max(1).astype(f32)
    out = [start]
    c = x[start]
    d = d2(xs[:, 0], xs[:, 1], xs[:, 2], c[0], c[1], c[2])
    dmin = np.where(real & (d < dmin), d, dmin)
    rounds, sizes = 0, []
    while len(out) < npoint:
        v = dmin.reshape(G, S)
        p = pid.reshape(G, S)
        # group best by (value desc, index asc) and the second largest value
        key_best = np.lexsort((p, -v), axis=1)[:, 0]
        cv = v[np.arange(G), key_best].copy()
        cp = p[np.arange(G), key_best].copy()
        srt = np.sort(v, 1)
        ub = srt[:, -2].copy()
        cxyz = xs.reshape(G, S, 3)[np.arange(G), key_best].copy()
        # walker: lane l holds groups l, l+64, ...; it lists its best, the rest bound by T
        listed = np.zeros(G, bool)
        T = f32(-1)
        for l in range(lanes):
            gs = np.arange(l, G, lanes)
            if len(gs) == 0:
                continue
            bi = gs[np.lexsort((cp[gs], -cv[gs]))[0]]
            listed[bi] = True
            rest = gs[gs != bi]
            if len(rest):
                T = max(T, cv[rest].max())
        alive = listed.copy()
        acc = []
        while len(out) + len(acc) < npoint:
            idx = np.flatnonzero(alive)
            if len(idx) == 0:
                break
            j = idx[np.lexsort((cp[idx], -cv[idx]))[0]]
            UB = max(T, ub[listed].max())
            if acc and not (cv[j] > UB):
                break
            acc.append(j)
            alive[j] = False
            cc = cxyz[j]
            # exact candidate updates and rounding-safe bound updates
            dd = d2(cxyz[:, 0], cxyz[:, 1], cxyz[:, 2], cc[0], cc[1], cc[2])
            cv = np.where(dd < cv, dd, cv)
            ub = np.minimum(ub, maxd2(gl, gh, cc))
            T = min(T, maxd2(gl, gh, cc)[~listed].max()) if (~listed).any() else T
        for j in acc:
            out.append(int(cp[j]))
            cc = cxyz[j]
            d = d2(xs[:, 0], xs[:, 1], xs[:, 2], cc[0], cc[1], cc[2])
            dmin = np.where(real & (d < dmin), d, dmin)
        rounds += 1
        sizes.append(len(acc))
    return np.array(out[:npoint]), rounds, np.array(sizes)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    npoint = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    rng = np.random.default_rng(0)
    cases = {
        "uniform": rng.uniform(-1, 1, (N, 3)).astype(f32),
        "dyadic-ties": (rng.integers(-8, 9, (N, 3)) / 8).astype(f32),
        "duplicates": np.repeat(rng.uniform(-1, 1, (N // 4, 3)).astype(f32), 4, 0),
        "surface": (lambda u: (u / np.linalg.norm(u, axis=1, keepdims=True)).astype(f32))(rng.normal(size=(N, 3))),
    }
    for name, x in cases.items():
        start = int(rng.integers(0, N))
        want = serial_fps(x, npoint, start)
        got, rounds, sizes = batched_fps(x, npoint, start)
        ok = np.array_equal(want, got)
        print(f"{name:12s} N={N} npoint={npoint}: exact={ok} rounds={rounds} mean batch={sizes.mean():.2f} "
              f"last-half={sizes[len(sizes) // 2:].mean():.2f}")
        assert ok, (name, np.flatnonzero(want != got)[:5])


if __name__ == "__main__":
    main()
