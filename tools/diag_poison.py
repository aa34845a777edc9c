"""Diagnostic: does any FE kernel read LDS or registers it never wrote?  Runs tests/test_gpu_dist.py's
batch once clean and then with tools/poison (every CU's LDS and a wave's VGPRs filled with a bit
pattern) launched on the same stream right before each set-abstraction table and FE-head launch.
A kernel whose output then changes reads state left behind by earlier work on the CU -- which in
one process is its own previous workgroups' (so repeats agree), but another process's kernels
when two share the GPU.

    python tools/diag_poison.py [--pkg DIR]
"""
import argparse
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import diag_shard_ranks as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pkg", default=os.path.join(S.ROOT, "deepvcp-pointcloud-registration_amd"))
    ap.add_argument("--lib", default=os.path.join(HERE, "poison", "libpoison.so"))
    a = ap.parse_args()
    S._paths(a.pkg)
    import torch
    from dvcp import ops
    lib = ctypes.CDLL(a.lib)
    lib.dvcp_poison.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    state = {"pattern": None}
    for name in ("sa_group_mlp", "sa_group_mlp_rows", "fe_head", "fe_head_rows", "ball_query"):
        orig = getattr(ops, name, None)
        if orig is None:
            continue

        def wrap(*args, _orig=orig, **kw):
            if state["pattern"] is not None:
                rc = lib.dvcp_poison(state["pattern"], ctypes.c_void_p(sink.data_ptr()),
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                assert rc == 0, rc
            return _orig(*args, **kw)
        setattr(ops, name, wrap)
    lib.dvcp_spin.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    delay = {"fps": 0, "side": 0}

    def spin(ticks):
        if ticks:
            assert lib.dvcp_spin(ticks, ctypes.c_void_p(sink.data_ptr()),
                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    orig_fps = ops.fps

    def fps(*args, **kw):
        spin(delay["fps"])
        return orig_fps(*args, **kw)
    ops.fps = fps
    for name in ("sa_group_mlp", "sa_group_mlp_rows", "ball_query"):
        orig = getattr(ops, name)

        def wrap2(*args, _orig=orig, **kw):
            spin(delay["side"])
            return _orig(*args, **kw)
        setattr(ops, name, wrap2)
    S._instrument()
    model, data, starts = S._setup("default")
    model.to(dev)
    clean = S._run(model, data, starts, dev, 0, S.P_TOTAL)
    again = S._run(model, data, starts, dev, 0, S.P_TOTAL)
    S.compare(clean, [again], "clean run twice")
    # shift the main stream's FPS launches or the side stream's tables by 0.5-5 ms (100 MHz ticks)
    for key, ticks in (("fps", 50000), ("fps", 200000), ("fps", 500000), ("side", 50000), ("side", 200000),
                       ("side", 500000)):
        delay.update(fps=0, side=0)
        delay[key] = ticks
        dirty = S._run(model, data, starts, dev, 0, S.P_TOTAL)
        S.compare(clean, [dirty], f"delay {key} {ticks / 1e5:.1f} ms")
        sys.stdout.flush()
    delay.update(fps=0, side=0)
    for pat in (0x7FC00000, 0x4B000000, 0x00000000, 0xBF800000):
        state["pattern"] = pat
        dirty = S._run(model, data, starts, dev, 0, S.P_TOTAL)
        S.compare(clean, [dirty], f"poison {pat:#010x}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
