"""CPU model of the partitioned `$-` root exchange (kernels.hip ws_roots: k_rt_prefix,
k_rt_offsets, k_rt_pack, the RCCL send/recv, and k_bits_compact's lookup).

A hop sends only the roots of the vertices whose bits it sends, packed per destination rank in
bit order.  The offsets come from popcount prefixes: per 64-bit word within a block of RW_BLOCK
words (k_rt_prefix), the blocks' totals scanned within each rank segment (k_rt_offsets), and the
per-rank counts scanned into displacements.  The owner finds a vertex's root at
disp_recv[q] + block offset + word prefix + popcount of the word's lower bits, for the highest
rank q whose segment has the vertex's bit (the reference's backtracker is last-write-wins).
This model restates that arithmetic on random bitmaps and checks every root comes back."""
import numpy as np
import pytest

RW_BLOCK = 1024   # kernels.hip: bitmap words per prefix block (npad / 64 is a multiple of it)


def _rank_side(send_bits, world, npad):
    """One rank's k_rt_prefix + k_rt_offsets over its send and received bitmaps."""
    seg_words = npad // 64
    nwords = world * seg_words
    pc = send_bits.reshape(-1, 64).sum(axis=1)
    pre = np.zeros(nwords, np.int64)
    bsum = np.zeros(nwords // RW_BLOCK, np.int64)
    for b in range(nwords // RW_BLOCK):
        blk = pc[b * RW_BLOCK:(b + 1) * RW_BLOCK]
        pre[b * RW_BLOCK:(b + 1) * RW_BLOCK] = np.cumsum(blk) - blk
        bsum[b] = blk.sum()
    spb = seg_words // RW_BLOCK
    boff = np.zeros_like(bsum)
    cnt = np.zeros(world, np.int64)
    for q in range(world):
        seg = bsum[q * spb:(q + 1) * spb]
        boff[q * spb:(q + 1) * spb] = np.cumsum(seg) - seg
        cnt[q] = seg.sum()
    disp = np.cumsum(cnt) - cnt
    return pre, boff, cnt, disp


@pytest.mark.parametrize("world,density", [(2, 0.3), (4, 0.02), (8, 0.001), (8, 0.5)])
def test_packed_roots_come_back(world, density):
    rng = np.random.default_rng(world * 1000 + int(density * 1000))
    npad = 65536
    seg_words = npad // 64
    send = [rng.random(world * npad) < density for _ in range(world)]
    bt_out = [rng.integers(1, 1 << 50, world * npad) for _ in range(world)]
    packs, cnts, disps = [], [], []
    for r in range(world):
        pre, boff, cnt, disp = _rank_side(send[r], world, npad)
        pack = np.zeros(cnt.sum(), np.int64)
        words = np.nonzero(send[r].reshape(-1, 64).any(axis=1))[0]
        for w in words:   # k_rt_pack: the set bits of word w in bit order
            at = disp[w // seg_words] + boff[w // RW_BLOCK] + pre[w]
            for b in np.nonzero(send[r][w * 64:(w + 1) * 64])[0]:
                pack[at] = bt_out[r][w * 64 + b]
                at += 1
        packs.append(pack)
        cnts.append(cnt)
        disps.append(disp)
    for r in range(world):
        # received bitmap: segment q = rank q's send segment r; its counts are the senders'
        recv = np.concatenate([send[q][r * npad:(r + 1) * npad] for q in range(world)])
        pre, boff, cnt, disp = _rank_side(recv, world, npad)
        assert [cnts[q][r] for q in range(world)] == list(cnt)   # host counts agree (alltoallv)
        buf = np.zeros(cnt.sum(), np.int64)
        for q in range(world):
            buf[disp[q]:disp[q] + cnt[q]] = packs[q][disps[q][r]:disps[q][r] + cnts[q][r]]
        for v in rng.integers(0, npad, 500):   # k_bits_compact: the highest sending rank's root
            word, bit = v // 64, v % 64
            want = None
            for q in range(world - 1, -1, -1):
                if send[q][r * npad + v]:
                    want = bt_out[q][r * npad + v]
                    break
            if want is None:
                continue
            for q in range(world - 1, -1, -1):
                rw = q * seg_words + word
                bits = recv[rw * 64:rw * 64 + 64]
                if bits[bit]:
                    at = disp[q] + boff[rw // RW_BLOCK] + pre[rw] + int(bits[:bit].sum())
                    assert buf[at] == want
                    break
