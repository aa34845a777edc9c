"""CPU checks of the batch-statistics BatchNorm host logic (dvcp/batchnorm.py): the pack layout
the HIP kernels read, the running-statistics update against torch's BatchNorm2d in training
mode, and the chunked weight-gradient GEMM (no GPU: the kernels themselves are checked in
tests/test_gpu_train.py)."""
import pytest
import torch


def test_pack_layout_matches_library():
    """Per layer W | bias | scale | shift | mean | istd | A/M | B/M, sized as the library says."""
    from dvcp import batchnorm, ops
    for chans in ([3, 16, 16, 32], [6, 16, 16, 32], [35, 32, 64], [67, 64, 64]):
        offs, total = batchnorm._layer_offsets(chans)
        assert total == ops.sa_bn_pack_floats(chans)
        o = 0
        for (off, cin, cout), a, b in zip(offs, chans[:-1], chans[1:]):
            assert (off, cin, cout) == (o, a, b)
            o += b * a + 7 * b


@pytest.mark.parametrize("momentum", [0.1, 0.3, None])
def test_running_update_matches_batchnorm2d(momentum):
    """_update_running(bn, batch mean, biased var, M) == what BatchNorm2d.forward in train mode
    does to running_mean / running_var / num_batches_tracked (unbiased variance, momentum or the
    cumulative average when momentum is None), over two batches."""
    from dvcp import batchnorm
    g = torch.Generator().manual_seed(3)
    ref = torch.nn.BatchNorm2d(8, momentum=momentum)
    mine = torch.nn.BatchNorm2d(8, momentum=momentum)
    for _ in range(2):
        x = torch.randn(4, 8, 5, 7, generator=g) * 3 + 1
        ref.train()(x)
        z = x.transpose(0, 1).reshape(8, -1).double()
        M = z.shape[1]
        mean = z.mean(1)
        var = ((z - mean[:, None]) ** 2).mean(1)
        batchnorm._update_running(mine, mean, var, M)
    torch.testing.assert_close(mine.running_mean, ref.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mine.running_var, ref.running_var, rtol=1e-5, atol=1e-6)
    assert int(mine.num_batches_tracked) == int(ref.num_batches_tracked) == 2


@pytest.mark.parametrize("nch,K", [(1, 64), (3, 4096), (5, 1000)])
def test_chunked_gemm(nch, K):
    """_gemm_nt over (nch, m, K) / (nch, n, K) chunked row tables == the plain product over the
    nch * K entries."""
    from dvcp.batchnorm import _gemm_nt
    g = torch.Generator().manual_seed(nch * K)
    a = torch.randn(nch, 16, K, generator=g)
    b = torch.randn(nch, 17, K, generator=g)
    want = a.permute(1, 0, 2).reshape(16, -1).double() @ b.permute(1, 0, 2).reshape(17, -1).double().t()
    got = _gemm_nt(a, b)
    assert got.dtype == torch.float64
    torch.testing.assert_close(got, want, rtol=0, atol=1e-3)
