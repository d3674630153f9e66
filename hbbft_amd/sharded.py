"""Validator-sharded broadcast simulation over several GPUs.

The N simulated validators are split into G contiguous blocks of R = ceil(N/G),
one block per rank (one GPU per rank): rank g hosts validators
[g*R, min((g+1)*R, N)).  Every rank proposes `count` broadcast instances per
step; local instance i of rank g has proposer g*R + (i mod |block g|).

One step follows the messages of /root/reference/src/broadcast/broadcast.rs:

1. proposer rank: frame + encode + Merkle tree + N proofs (send_shards,
   170-225), all through libhbrbc.so.
2. Value (212-222): shard j with its proof goes to validator j, i.e. to rank
   owner(j).  Over all instances that is an all-to-all of [G][count][R] shard
   rows plus their digests (RCCL over xGMI when the group is NCCL).  The root
   travels inside every proof; the roots are all-gathered (the Ready/EchoHash
   fan-out of 32-byte digests).
3. every validator validates its Value (handle_value -> validate_proof,
   254 / 604-606): one Proof::validate per (instance, validator).
4. Echo (send_echo_left, 413-425): validator j sends its shard and proof to the
   N-f nodes on its left.  The simulated receiver of each instance is the
   proposer's own node p, which gets Echoes from every validator except its
   f right-hand neighbours p+1..p+f (right_nodes, 476-485) and except
   validators whose Value failed validation (they send no Echo, 254-256).
   The Echo rows go back to the proposer's rank: a second all-to-all.
5. the receiver decodes (compute_output -> decode_from_shards, 526-601):
   reconstruct, re-tree, root compare, unframe.

What is not re-run: the receiver's Proof::validate of each Echo (291)
repeats step 3's computation on the same bytes, proof and index, and the
other N-1 nodes' decodes reproduce the same payload from the same codeword;
both are pure functions of identical inputs, so each is computed once.

Layouts (row = one shard of `stride` bytes):
  proposer slab   [count][G*R][stride]   rows >= N are padding (zeroed)
  Value send/recv [G][count][R][stride]  block d of send = rows d*R.. of every
                                         local instance; block s of recv =
                                         this rank's rows of rank s's instances
  Echo recv       [G][count][R][stride]  block v = rows v*R.. of every local
                                         instance, as validated on rank v
The regrouping is a plain strided copy done by torch (layout plumbing); every
byte of shard, digest and payload data is computed by the HIP kernels.
"""
import torch

from . import RbcBatch, shard_len


# ------------------------------------------------------------------ topology --
class Topology:
    """N validators over `world` ranks in contiguous blocks of R."""

    def __init__(self, n, world):
        if world < 1 or world > n:
            raise ValueError("need 1 <= world (%d) <= n (%d)" % (world, n))
        self.n, self.world = n, world
        self.f = (n - 1) // 3
        self.rpg = -(-n // world)
        if (world - 1) * self.rpg >= n:
            raise ValueError("n=%d does not give every one of %d ranks a validator" % (n, world))
        self.npad = self.rpg * world

    def validators(self, rank):
        return range(rank * self.rpg, min((rank + 1) * self.rpg, self.n))

    def owner(self, j):
        return j // self.rpg

    def proposers(self, rank, count):
        """Proposer (validator index) of each local instance of `rank`."""
        vs = self.validators(rank)
        return [vs[i % len(vs)] for i in range(count)]

    def echo_received(self, proposers, device=None):
        """[count, n] bool: the receiver p gets an Echo from every validator but
        its f right-hand neighbours p+1..p+f (broadcast.rs:476-485)."""
        p = torch.as_tensor(proposers, dtype=torch.int64, device=device).view(-1, 1)
        j = torch.arange(self.n, dtype=torch.int64, device=device).view(1, -1)
        d = (j - p) % self.n
        return ~((d >= 1) & (d <= self.f))


# ---------------------------------------------------------- layout helpers ---
def pack_rows(slab, world, rpg, out):
    """[count][world*rpg][...] -> [world][count][rpg][...] (destination-major)."""
    count = slab.shape[0]
    out.copy_(slab.view(count, world, rpg, *slab.shape[2:]).transpose(0, 1))
    return out


def unpack_rows(buf, out):
    """[world][count][rpg][...] -> [count][world*rpg][...] (inverse of pack_rows)."""
    world, count, rpg = buf.shape[:3]
    out.view(count, world, rpg, *buf.shape[3:]).copy_(buf.transpose(0, 1))
    return out


# ---------------------------------------------------------------- exchange ---
class DistExchange:
    """all-to-all / all-gather over a torch.distributed group.  With NCCL
    (= RCCL on ROCm) the device buffers go straight over xGMI; with gloo
    (CPU tests, several ranks sharing one GPU) device tensors are staged
    through host memory."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.staged = dist.get_backend(group) != "nccl"

    def all_to_all(self, out, inp, async_op=False):
        """out[s] on this rank = inp[rank] on rank s (dim 0 = ranks).  With
        async_op (NCCL only) returns a handle; wait() makes torch's current
        stream wait for it, so the copy overlaps whatever is queued meanwhile."""
        assert out.shape[0] == self.world and inp.shape[0] == self.world
        if self.world == 1:
            if out.data_ptr() != inp.data_ptr():
                out.copy_(inp)
            return None
        if self.staged and out.is_cuda:
            o, i = out.cpu(), inp.cpu()
            self.dist.all_to_all_single(o, i, group=self.group)
            out.copy_(o)
            return None
        return self.dist.all_to_all_single(out, inp, group=self.group,
                                           async_op=async_op and not self.staged)

    def all_gather(self, out, inp, async_op=False):
        """out[s] = inp of rank s."""
        if self.world == 1:
            out[0].copy_(inp)
            return None
        if self.staged:
            parts = [torch.empty_like(inp, device="cpu") for _ in range(self.world)]
            self.dist.all_gather(parts, inp.cpu(), group=self.group)
            out.copy_(torch.stack(parts))
            return None
        return self.dist.all_gather_into_tensor(out, inp.contiguous(), group=self.group,
                                                async_op=async_op)


def wait_all(handles):
    for h in handles:
        if h is not None:
            h.wait()


class SoloExchange:
    """The exchange of a one-rank run (no process group): every collective is
    the identity, and ShardedBroadcast aliases its buffers so nothing moves."""

    world, rank = 1, 0

    def all_to_all(self, out, inp, async_op=False):
        if out.data_ptr() != inp.data_ptr():
            out.copy_(inp)

    def all_gather(self, out, inp, async_op=False):
        out[0].copy_(inp)


def loopback_all_to_all(outs, ins):
    """The all-to-all of `len(ins)` virtual ranks living in one process:
    outs[d][s] = ins[s][d]."""
    for d, o in enumerate(outs):
        for s, i in enumerate(ins):
            o[s].copy_(i[d])


# --------------------------------------------------------------- one rank ---
class ShardedBroadcast:
    """The per-rank state of the validator-sharded simulation: `count` local
    proposals of `plen` bytes per step on `device`."""

    def __init__(self, n, count, plen, rank, world, device=0):
        self.topo = t = Topology(n, world)
        self.rank, self.world, self.count, self.plen = rank, world, count, plen
        self.rb = rb = RbcBatch(n, t.f, device=device)
        dev = rb.device
        self.device = dev
        self.S = S = shard_len(plen, rb.k)
        self.stride = stride = rb.stride_for(S)
        ds = max(rb.dslots, 1)
        G, R, C = world, t.rpg, count
        u8 = dict(dtype=torch.uint8, device=dev)
        self.proposers = t.proposers(rank, C)
        # proposer side
        self.slab = torch.zeros((C, t.npad, stride), **u8)
        self.nodes = rb.alloc_nodes(C)
        self.digests = torch.zeros((C, n, ds, 32), **u8)
        self.ndig = torch.zeros((C, n), **u8)
        # Value exchange (rows R per destination; G == 1 aliases, no copy)
        if G == 1:
            self.send_sh = self.slab.view(1, C, R, stride)
        else:
            self.send_sh = torch.empty((G, C, R, stride), **u8)
        self.send_dg = torch.zeros((G, C, R, ds * 32 + 16), **u8)   # digests ++ ndig ++ pad
        self.dg_flat = torch.zeros((C, t.npad, ds * 32 + 16), **u8)
        self.recv_sh = self.send_sh if G == 1 else torch.empty_like(self.send_sh)
        self.recv_dg = self.send_dg if G == 1 else torch.empty_like(self.send_dg)
        self.roots_all = torch.empty((G, C, 32), **u8)
        # validator side: the claimed/expected index of every received row
        idx = torch.arange(rank * R, (rank + 1) * R, dtype=torch.int32, device=dev)
        self.recv_idx = idx.view(1, 1, R).expand(G, C, R).contiguous()
        self.ok_v = torch.zeros((G, C, R), **u8)
        self.v_digests = torch.empty((G, C, R, ds, 32), **u8)
        self.v_ndig = torch.empty((G, C, R), **u8)
        # Echo exchange back to the proposer's rank
        self.echo_sh = self.recv_sh if G == 1 else torch.empty_like(self.recv_sh)
        self.echo_ok = self.ok_v if G == 1 else torch.empty_like(self.ok_v)
        # receiver side
        self.dec_slab = self.slab if G == 1 else torch.zeros((C, t.npad, stride), **u8)
        self.echo_mask = t.echo_received(self.proposers, device=dev).to(torch.uint8)
        self.present = torch.empty((C, n), **u8)
        self.nodes2 = rb.alloc_nodes(C)
        self.out = torch.zeros((C, max(16, (rb.k * S + 15) // 16 * 16)), **u8)
        self.plen_out = torch.zeros(C, dtype=torch.int32, device=dev)
        self.status = torch.zeros(C, dtype=torch.int32, device=dev)
        rb.reserve(C)

    # 1. proposer: frame, encode, tree, proofs -------------------------------
    def propose(self, payloads):
        rb, S = self.rb, self.S
        slab = self.slab[:, : self.topo.n]
        rb.frame_encode(payloads, self.plen, slab)
        rb.merkle(slab, S, self.nodes)
        rb.proofs(self.nodes, self.digests, self.ndig)

    def roots(self):
        return self.nodes[:, -1, :]

    # 2. Value messages ---------------------------------------------------------
    def pack_value(self):
        G, R, C = self.world, self.topo.rpg, self.count
        n, ds = self.topo.n, self.digests.shape[2]
        if G > 1:
            pack_rows(self.slab, G, R, self.send_sh)
        flat = self.dg_flat
        flat[:, :n, : ds * 32] = self.digests.view(C, n, ds * 32)
        flat[:, :n, ds * 32] = self.ndig
        pack_rows(flat, G, R, self.send_dg)

    def exchange_value(self, ex, async_op=False):
        """Value messages (+ the roots' all-gather); returns the handles."""
        self._roots = self.roots().contiguous()   # kept alive while in flight
        return [ex.all_to_all(self.recv_sh, self.send_sh, async_op),
                ex.all_to_all(self.recv_dg, self.send_dg, async_op),
                ex.all_gather(self.roots_all, self._roots, async_op)]

    # 3. validators validate their Values --------------------------------------
    def validate_values(self):
        G, R, C = self.world, self.topo.rpg, self.count
        ds = self.digests.shape[2]
        self.v_digests.view(G, C, R, ds * 32).copy_(self.recv_dg[..., : ds * 32])
        self.v_ndig.copy_(self.recv_dg[..., ds * 32])
        self.rb.validate_rows(self.recv_sh.view(G * C, R, self.stride), self.S, R,
                              self.recv_idx.view(G * C, R), self.v_digests.view(G * C, R, ds, 32),
                              self.v_ndig.view(G * C, R), self.roots_all.view(G * C, 32),
                              self.ok_v.view(G * C, R))

    # 4. Echo messages back to the proposer's rank ------------------------------
    def exchange_echo(self, ex, async_op=False):
        """Echo messages back to the proposers' ranks; returns the handles."""
        return [ex.all_to_all(self.echo_sh, self.recv_sh, async_op),
                ex.all_to_all(self.echo_ok, self.ok_v, async_op)]

    # 5. the receiver decodes ---------------------------------------------------
    def decode(self):
        G, n = self.world, self.topo.n
        if G > 1:
            unpack_rows(self.echo_sh, self.dec_slab)
        ok = self.echo_ok.transpose(0, 1).reshape(self.count, self.topo.npad)[:, :n]
        torch.mul(ok, self.echo_mask, out=self.present)
        self.rb.decode(self.dec_slab[:, :n], self.S, self.present, self.roots(), self.nodes2,
                       self.out, self.plen_out, self.status)

    def step(self, payloads, ex):
        self.propose(payloads)
        self.pack_value()
        self.exchange_value(ex)
        self.validate_values()
        self.exchange_echo(ex)
        self.decode()


def pipelined_step(subs, payloads, ex):
    """One step over several sub-batches (ShardedBroadcast objects on the same
    rank, payloads[i] for subs[i]) with every exchange in flight while the next
    sub-batch computes: propose all -> (Value of i overlaps propose of i+1) ->
    validate i while Value i+1 / Echo i-1 move -> decode i while Echo i+1
    moves.  With NCCL the collectives run on the communicator's stream and
    handle.wait() only orders torch's current stream after them."""
    n = len(subs)
    hv, he = [None] * n, [None] * n
    for i, sb in enumerate(subs):
        sb.propose(payloads[i])
        sb.pack_value()
        hv[i] = sb.exchange_value(ex, async_op=True)
    for i, sb in enumerate(subs):
        wait_all(hv[i])
        sb.validate_values()
        he[i] = sb.exchange_echo(ex, async_op=True)
    for i, sb in enumerate(subs):
        wait_all(he[i])
        sb.decode()
