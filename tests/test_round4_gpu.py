"""GPU tests of the round-4 kernels: the chunked planning sort against the one-workgroup sort,
the one-launch multi-tensor copy (HIP-graph slot refill), the in-kernel clock probe, and the
one-sided dense push that folds split-K weight-gradient planes on the way into the inboxes."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _kernels():
    from minips_amd._native import kernels

    return kernels()


def test_multi_copy_matches_copy(dev):
    k = _kernels()
    srcs = [torch.randn(1000, device=dev), torch.randint(0, 1 << 40, (777,), device=dev),
            torch.randn(33, 17, device=dev).to(torch.bfloat16), torch.randint(0, 255, (5,), dtype=torch.uint8,
                                                                                 device=dev),
            torch.randn(4096 * 8, device=dev)]
    dsts = [torch.zeros_like(s) for s in srcs]
    k.multi_copy(dsts, srcs)
    torch.cuda.synchronize()
    for d, s in zip(dsts, srcs):
        assert torch.equal(d, s)
    # more than one launch's worth of pairs
    many_s = [torch.randn(100 + i, device=dev) for i in range(20)]
    many_d = [torch.zeros_like(s) for s in many_s]
    k.multi_copy(many_d, many_s)
    torch.cuda.synchronize()
    assert all(torch.equal(d, s) for d, s in zip(many_d, many_s))


def test_clock_probe_reads_a_plausible_clock(dev):
    k = _kernels()
    out = torch.zeros(2, dtype=torch.int64, device=dev)
    k.clock_probe(out, 2000, 0)
    torch.cuda.synchronize()
    cycles, ticks = int(out[0]), int(out[1])
    assert ticks >= 2000 and cycles > 0
    mhz = cycles / ticks * 100.0
    assert 50.0 < mhz < 4000.0, mhz


def test_ps_push_dense_folds_slab_planes(dev):
    """grad slice + the sum of every plane of the regions inside it lands in the inbox slot; grad is
    cleared (one owner; the owner's inbox is this device's buffer)."""
    k = _kernels()
    S = 4096
    grad = torch.randn(S, device=dev)
    inbox = torch.zeros(64 + 4 * S + 256, dtype=torch.uint8, device=dev)
    ptrs = torch.tensor([inbox.data_ptr()], dtype=torch.int64, device=dev)
    data_off = 64
    regions = [(0, 512, 3), (1024, 1024, 6), (3000, 96, 1)]  # (offset, length, nsplit)
    slabs, expect = [], grad.clone()
    for off, ln, ns in regions:
        planes = torch.randn(ns * ln, device=dev)
        slabs.append((planes, ns, ln, off))
        expect[off: off + ln] += planes.view(ns, ln).sum(0)
    k.ps_push_dense(grad, ptrs, data_off, S, slabs)
    torch.cuda.synchronize()
    got = inbox[data_off: data_off + 4 * S].view(torch.float32)
    torch.testing.assert_close(got, expect, rtol=1e-5, atol=1e-5)
    assert float(grad.abs().max()) == 0.0
