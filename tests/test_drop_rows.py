"""hbrbc_drop_rows (include/hbrbc.h): the rows a receiver never got are
overwritten, whole slot, in the plain and the blocked layout; every other
byte is untouched; a decode after it rebuilds the rows exactly (the bench's
`erase` stage)."""
import numpy as np
import pytest
import torch

import hbbft_amd as hb
from oracle import pyoracle as orc


@pytest.mark.gpu
@pytest.mark.parametrize("n,count,stride", [(4, 3, 32), (64, 17, 11920), (250, 2, 49936),
                                            (16, 5, 16)])
def test_drop_rows_plain(n, count, stride):
    rb = hb.RbcBatch(n, device=0)
    g = torch.Generator().manual_seed(n * 1000 + count)
    slab = torch.randint(0, 256, (count, n, stride), dtype=torch.uint8, generator=g)
    present = (torch.rand((count, n), generator=g) < 0.6).to(torch.uint8)
    want = slab.clone()
    want[present == 0] = 0x3C
    d = slab.cuda()
    rb.drop_rows(d, present.cuda(), 0x3C)
    torch.cuda.synchronize()
    assert torch.equal(d.cpu(), want)


@pytest.mark.gpu
def test_drop_rows_blocked_layout():
    """Rows in blocks of R over G destination blocks ([G][count][R][stride],
    the validator-sharded slab): row j of instance i lives in block j // R."""
    n, G, count, stride = 10, 4, 3, 48
    R = -(-n // G)
    rb = hb.RbcBatch(n, device=0)
    g = torch.Generator().manual_seed(7)
    slab = torch.randint(0, 256, (G, count, R, stride), dtype=torch.uint8, generator=g)
    present = (torch.rand((count, n), generator=g) < 0.5).to(torch.uint8)
    want = slab.clone()
    for i in range(count):
        for j in range(n):
            if not present[i, j]:
                want[j // R, i, j % R] = 0x77
    d, p = slab.cuda(), present.cuda()
    hb._check(hb.lib().hbrbc_drop_rows(rb.coding.handle, d.data_ptr(), stride, R,
                                       count * R * stride, R * stride, p.data_ptr(), count, 0x77,
                                       None))
    torch.cuda.synchronize()
    assert torch.equal(d.cpu(), want)


@pytest.mark.gpu
def test_decode_after_drop_rows_matches_oracle():
    """Encode, drop f rows per instance, decode: rows, trees and payloads as
    the oracle's send_shards / decode."""
    n, f, count, plen = 16, 5, 6, 5000
    rb = hb.RbcBatch(n, f, device=0)
    S = hb.shard_len(plen, rb.k)
    stride = rb.stride_for(S)
    pays = np.stack([orc.gen_payload(77, i, plen) for i in range(count)])
    pt = torch.zeros((count, (plen + 15) // 16 * 16), dtype=torch.uint8)
    pt[:, :plen] = torch.from_numpy(pays)
    pt = pt.cuda()
    slab = torch.zeros((count, n, stride), dtype=torch.uint8, device="cuda")
    nodes = rb.alloc_nodes(count)
    rb.frame_encode(pt, plen, slab)
    rb.merkle(slab, S, nodes)
    ref = slab.clone()
    present = torch.stack([torch.from_numpy(orc.gen_present(77, i, n, f)) for i in range(count)])
    present = present.cuda()
    rb.drop_rows(slab, present)
    torch.cuda.synchronize()
    assert not torch.equal(slab, ref)
    roots = nodes[:, -1, :].contiguous()
    nodes2 = rb.alloc_nodes(count)
    out = torch.zeros((count, (rb.k * S + 15) // 16 * 16), dtype=torch.uint8, device="cuda")
    plen_out = torch.zeros(count, dtype=torch.int32, device="cuda")
    status = torch.zeros(count, dtype=torch.int32, device="cuda")
    rb.decode(slab, S, present, roots, nodes2, out, plen_out, status)
    torch.cuda.synchronize()
    assert (status.cpu() == 0).all() and (plen_out.cpu() == plen).all()
    assert torch.equal(slab, ref) and torch.equal(nodes2, nodes)
    for i in range(count):
        sh, nd = orc.send_shards(n, f, pays[i].tobytes())
        assert np.array_equal(out[i, :plen].cpu().numpy(), pays[i])
        assert np.array_equal(nodes[i].cpu().numpy(), nd)
