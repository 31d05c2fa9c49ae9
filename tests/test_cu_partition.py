"""CPU checks of the CU-partition mask arithmetic (utils/cu_partition.py)."""
import pytest

from pytorch_operator_1_amd.utils import cu_partition as cp


@pytest.mark.parametrize("layout", ["block", "stride"])
@pytest.mark.parametrize("parts", [1, 2, 3, 4, 8])
def test_partitions_disjoint_and_cover(layout, parts):
    n = 256
    seen = []
    for k in range(parts):
        bits = cp.mask_bits(k, parts, n, layout)
        assert abs(len(bits) - n / parts) < 1
        seen.append(set(bits))
    assert set().union(*seen) == set(range(n))
    assert sum(len(s) for s in seen) == n


def test_mask_words_roundtrip():
    bits = cp.mask_bits(1, 2, 256, "block")
    w = cp.mask_words(bits, 256)
    assert len(w) == 8 and w[:4] == [0] * 4 and w[4:] == [0xFFFFFFFF] * 4
    assert cp.words_bits(w) == bits
    assert cp.mask_words(cp.mask_bits(0, 2, 256, "stride"), 256) == [0x55555555] * 8
    with pytest.raises(ValueError):
        cp.mask_words([256], 256)
    with pytest.raises(ValueError):
        cp.mask_bits(2, 2, 256)


def test_decode_hw_id_and_summary():
    hw = (5 << 8) | (1 << 12) | (3 << 13) | (2 << 24)  # CU 5, SH 1, SE 3, queue 2
    f = cp.decode_hw_id(hw)
    assert (f["cu"], f["sh"], f["se"], f["queue"]) == (5, 1, 3, 2)
    assert cp.cu_key(7, hw) == (7, 3, 1, 5)
    s = cp.summarize([7, hw, 7, hw | 3, 0, 0])  # two waves on one CU (wave id differs), one elsewhere
    assert s["n_cus"] == 2 and s["cus_per_xcc"] == {0: 1, 7: 1} and s["queues"] == [0, 2]


def test_share_of_round_robin():
    # 8 local ranks on 2 GPUs: ranks 0,2,4,6 on GPU 0 as partitions 0..3 of 4
    assert [cp.share_of(r, 8, 2) for r in (0, 2, 4, 6)] == [(0, k, 4) for k in range(4)]
    assert cp.share_of(3, 8, 2) == (1, 1, 4)
    assert cp.share_of(0, 1, 1) == (0, 0, 1)
    assert cp.share_of(1, 2, 8) == (1, 0, 1)  # a GPU each: no partition
    assert cp.share_of(1, 3, 2) == (1, 0, 1) and cp.share_of(2, 3, 2) == (0, 1, 2)
