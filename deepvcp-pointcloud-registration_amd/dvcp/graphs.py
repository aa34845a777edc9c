"""One inference step captured as a HIP graph and replayed (torch.cuda.CUDAGraph over the C ABI's
stream-ordered launches; every entry point is capture-safe, include/dvcp.h).

A step is ``DeepVCP.forward`` + ``deepVCP_loss`` (+ the train.py:112-120 registration error) on
static input tensors: ``replay(starts)`` copies the step's seven FPS start vectors into the
graph's device buffer and launches the whole dependency graph -- ~60 kernels on the step's stream
and its side streams -- with one host call instead of one Python + ctypes call per kernel.  The
outputs are the graph's static tensors (overwritten by the next replay).  The device error words
a step raises (the voxel grid's, the split FPS's) are collected at capture and checked after
each replay, as the eager path checks them (dvcp._lib.defer_flag_check).

Replays equal the eager forward on the same inputs bit for bit (tests/test_gpu_e2e.py
test_captured_step_equals_eager).  The model's weights must not change after capture (the packed
parameters are captured by address).
"""
import torch

from . import _lib
from .deepVCP_loss import deepVCP_loss
from .ops import registration_error


class CapturedStep:
    def __init__(self, model, src, tgt, R_gt, t_gt, alpha=0.5, stream=None, starts=None):
        """``src``, ``tgt`` (B, C_in, N), ``R_gt`` (B, 3, 3) fp64, ``t_gt`` (B, 3, 1) fp64: device
        tensors the graph reads in place (refill them between replays to run other pairs).
        ``stream``: the stream the step is captured on and replayed on (default: a new one).
        ``starts`` (7, B): the FPS starts of the warm-up run (drawn like the reference if None)."""
        if _lib.EVENT_LOG is not None:
            raise RuntimeError("dvcp.graphs: per-kernel event logging cannot be captured")
        dev = src.device
        self.model, self.src, self.tgt, self.R_gt, self.t_gt, self.alpha = model, src, tgt, R_gt, t_gt, alpha
        self.stream = stream if stream is not None else torch.cuda.Stream(device=dev)
        B = src.shape[0]
        if starts is None:
            starts = model.draw_starts(B, src.shape[2], tgt.shape[2])
        self.starts = torch.empty(7, B, dtype=torch.int64, device=dev)
        # pinned staging for host starts: a ring, each slot reused only after its copy has run
        self._host = [torch.empty(7, B, dtype=torch.int64, pin_memory=True) for _ in range(4)]
        self._host_ev = [None] * 4
        self._slot = 0
        self.t_init = torch.zeros(1, 3)
        cur = torch.cuda.current_stream(dev)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self.starts.copy_(starts)
            self._body()            # warm-up: packed parameters, side streams, allocator pools
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        _lib._CAPTURED_FLAGS = []
        try:
            with torch.cuda.graph(self.graph, stream=self.stream):
                self.out = self._body()
            self.flags = _lib._CAPTURED_FLAGS
        finally:
            _lib._CAPTURED_FLAGS = None

    def _body(self):
        with torch.no_grad():
            kp, vcp = self.model(self.src, self.tgt, self.R_gt, self.t_init, starts=self.starts)
            _, R, t = deepVCP_loss(kp, vcp, self.R_gt, self.t_gt, self.alpha)
            rot, trans = registration_error(R, t, self.R_gt, self.t_gt)
        return R, t, rot, trans

    def replay(self, starts):
        """Run the captured step with these FPS starts ((7, B) int64, host or device) on the
        step's stream; returns the static outputs (R, t, rotation error, translation error)."""
        with torch.cuda.stream(self.stream):
            if starts.is_cuda:
                self.starts.copy_(starts, non_blocking=True)
            else:
                k = self._slot
                self._slot = (k + 1) % len(self._host)
                if self._host_ev[k] is not None:
                    self._host_ev[k].synchronize()
                self._host[k].copy_(starts)
                self.starts.copy_(self._host[k], non_blocking=True)
                self._host_ev[k] = torch.cuda.Event()
                self._host_ev[k].record(self.stream)
            self.graph.replay()
            for what, flag in self.flags:
                _lib.defer_flag_check(what, flag)
        return self.out
