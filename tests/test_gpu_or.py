"""fm_or_bits (csrc/shard.hip), the exchange step of doc-range sharding
(SURVEY §8e): the OR of P shards' bit-packed rows, as uint8 [B, V] 0/1 or as
packed words, against torch on random words -- both kernel shapes (16-B loads
when rows hold a multiple of 4 words, word loads otherwise), part counts
around the 8-load batch, vocab tails that end inside a 16-token chunk, row
strides wider than the vocab and a misaligned output."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def _expect(parts, V):
    import torch

    x = parts[0].clone()
    for p in parts[1:]:
        x |= p
    bits = ((x.to(torch.int64) & 0xFFFFFFFF).unsqueeze(-1) >> torch.arange(32, device=x.device)) & 1
    return x, bits.reshape(x.shape[0], -1)[:, :V].to(torch.uint8)


@pytest.mark.parametrize("P,B,V", [(1, 3, 17), (8, 5, 128256), (9, 4, 128256), (3, 7, 8192 * 2 + 33),
                                   (16, 2, 32 * 4 * 256), (5, 6, 100), (2, 1, 32 * 3 + 5), (11, 3, 151936)])
def test_or_bits_vs_torch(dev, P, B, V):
    import torch

    from fmidx.sharding import or_bits

    W = (V + 31) // 32
    g = torch.Generator(device="cpu").manual_seed(P * 1000 + V)
    # sparse words (most rows of a real step are nearly empty) and dense ones
    raw = torch.randint(-(1 << 31), 1 << 31, (P, B, W), generator=g, dtype=torch.int64)
    keep = torch.rand((P, B, W), generator=g) < 0.3
    parts = torch.where(keep, raw, torch.zeros_like(raw)).to(torch.int32).to(dev).contiguous()
    words, want = _expect(parts, V)
    assert torch.equal(or_bits(parts, V), want)
    assert torch.equal(or_bits(parts, V, unpack=False), words)
    # a row stride wider than the vocab, and an output that starts 1 byte into its allocation
    wide = torch.full((B, V + 48), 7, dtype=torch.uint8, device=dev)
    or_bits(parts, V, out=wide[:, :V])
    assert torch.equal(wide[:, :V], want) and bool((wide[:, V:] == 7).all())
    skew = torch.full((B, V + 17), 7, dtype=torch.uint8, device=dev)
    or_bits(parts, V, out=skew[:, 1:V + 1])
    assert torch.equal(skew[:, 1:V + 1], want) and bool((skew[:, 0] == 7).all())
    wide_w = torch.full((B, W + 4), 5, dtype=torch.int32, device=dev)
    or_bits(parts, V, out=wide_w[:, :W], unpack=False)
    assert torch.equal(wide_w[:, :W], words) and bool((wide_w[:, W:] == 5).all())


def test_or_bits_rejects_short_rows(dev):
    import torch

    from fmidx import FMIndexError
    from fmidx.sharding import or_bits

    parts = torch.zeros((2, 3, 4), dtype=torch.int32, device=dev)
    with pytest.raises(FMIndexError):
        or_bits(parts, 200)                      # 4 words cannot hold 200 tokens
    with pytest.raises(ValueError):
        or_bits(parts, 100, out=torch.empty((3, 100), dtype=torch.uint8, device=dev)[:, :50])
    np.testing.assert_array_equal(or_bits(parts, 100).cpu().numpy(), np.zeros((3, 100), np.uint8))
