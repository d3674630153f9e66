"""Validator-sharded broadcast simulation over several GPUs.

The N simulated validators are split into G contiguous blocks of R = ceil(N/G),
one block per rank (one GPU per rank): rank g hosts validators
[g*R, min((g+1)*R, N)).  Every rank proposes `count` broadcast instances per
step; local instance i of rank g has proposer g*R + (i mod |block g|).

One step follows the messages of /root/reference/src/broadcast/broadcast.rs:

1. proposer rank: frame + encode + Merkle tree + N proofs (send_shards,
   170-225).  The encoder writes the shard slab destination-major,
   [G][count][R][stride] (a blocked row layout of libhbrbc, hbrbc.h
   "*_rows"), so block d is already the contiguous chunk that goes to rank d.
2. Value (212-222): shard j with its proof goes to validator j, i.e. to rank
   owner(j): one all-to-all of the slab (RCCL over xGMI when the group is
   NCCL), one of the digests; the roots are all-gathered (the 32-byte
   Ready/EchoHash fan-out).
3. every validator validates its Value (handle_value -> validate_proof,
   254 / 604-606): one Proof::validate per (instance, validator), which also
   yields the row's Merkle leaf.
4. Echo (send_echo_left, 413-425): validator j sends its shard and proof to
   every node but its f right-hand neighbours.  Since every rank hosts
   receivers, that fan-out is an all-gather of the validated rows: afterwards
   every rank holds every row of every instance, [G][G*count][R][stride],
   which is again a blocked layout -- decoded in place, no unpacking.
5. every rank decodes every instance (compute_output -> decode_from_shards,
   526-601) for the receivers it hosts.

Per-GPU dedup (validate and decode are pure functions, so
identical calls on one GPU are computed once; the bench reports faithful and
executed counts):
  * the receivers of rank g all decode the same codewords; the rank decodes
    each instance once, as its first validator r0 = g*R sees it: every Echo
    but those of r0's right-hand neighbours r0+1..r0+f (476-485), and none
    from a validator whose Value failed (it sends no Echo, 254-256);
  * rank g validates each Echo it receives once (291); rows of its own
    validators were validated as their Values in step 3 (same bytes, proof,
    index and root);
  * the decode reuses those validations' leaf digests (hbrbc_decode_rows
    known_leaves): only the rows reconstruct rebuilds are hashed again.
With global-dedup instance mode (bench.py default) the unit of work is one
decode per instance; here it is one decode per instance per rank, which is
what a node of a G-GPU deployment must do.
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
        # rows_per_block of the slabs (0: plain shard-major layout)
        self.rows_per_block = self.rpg if world > 1 else 0

    def validators(self, rank):
        return range(rank * self.rpg, min((rank + 1) * self.rpg, self.n))

    def owner(self, j):
        return j // self.rpg

    def proposers(self, rank, count):
        """Proposer (validator index) of each local instance of `rank`."""
        vs = self.validators(rank)
        return [vs[i % len(vs)] for i in range(count)]

    def receiver(self, rank):
        """The validator whose view rank `rank` decodes with (its first)."""
        return rank * self.rpg

    def receiver_present(self, rank):
        """n flags: the Echoes receiver(rank) gets -- all but its f right-hand
        neighbours r0+1..r0+f (broadcast.rs:476-485)."""
        r0 = self.receiver(rank)
        right = {(r0 + d) % self.n for d in range(1, self.f + 1)}
        return [0 if j in right else 1 for j in range(self.n)]

    def echo_rows(self, rank):
        """Rows rank `rank` validates as Echoes: received by its receiver and
        sent by validators of other ranks."""
        pres = self.receiver_present(rank)
        return [j for j in range(self.n) if pres[j] and self.owner(j) != rank]


# ---------------------------------------------------------------- exchange ---
class _StagedWork:
    """Handle of a host-staged (gloo) collective issued with async_op: wait()
    waits for the gloo work, then copies the host result into the device
    tensor on the current stream -- the same point at which an NCCL handle's
    wait() makes the current stream wait for the RCCL kernel, so the staged
    rehearsal runs the handle/event ordering of the RCCL path."""

    def __init__(self, work, host_out, out):
        self.work, self.host_out, self.out = work, host_out, out

    def wait(self):
        self.work.wait()
        if self.out is not None:
            self.out.copy_(self.host_out())
        self.work = self.out = None


class DistExchange:
    """all-to-all / all-gather over a torch.distributed group.  With NCCL
    (= RCCL on ROCm) the device buffers go straight over xGMI; with gloo
    (CPU tests, several ranks sharing one GPU) device tensors are staged
    through host memory.  Both backends return a handle when async_op is set
    (wait() = the current stream / host waits for the exchange, and for gloo
    the copy back to the device), so the pipelined schedule is the same code
    on both.  Every call is counted per collective name: calls and bytes this
    rank sends (bench line, `exchange.per_rank`).  `loop`: a one-rank group
    still issues its collectives (tests/rccl_one_rank.py runs the RCCL calls
    on the one GPU of a test box); without it a one-rank group copies."""

    def __init__(self, group=None, loop=False):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.loop = loop
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        self.staged = self.backend != "nccl"
        self.stats = {}

    def _count(self, name, nbytes):
        e = self.stats.setdefault(name, {"calls": 0, "bytes_sent": 0})
        e["calls"] += 1
        e["bytes_sent"] += int(nbytes)

    def reset_stats(self):
        self.stats = {}

    def all_to_all(self, out, inp, async_op=False, name="all_to_all"):
        """out[s] on this rank = inp[rank] on rank s (dim 0 = ranks).  With
        async_op returns a handle whose wait() makes the current stream wait."""
        assert out.shape[0] == self.world and inp.shape[0] == self.world
        assert out.is_contiguous() and inp.is_contiguous()
        if self.world == 1 and not self.loop:
            if out.data_ptr() != inp.data_ptr():
                out.copy_(inp)
            return None
        # this rank keeps chunk `rank` and sends the other world - 1
        self._count(name, inp.numel() * inp.element_size() * (self.world - 1) // self.world)
        if self.staged and out.is_cuda:
            o, i = torch.empty(out.shape, dtype=out.dtype), inp.cpu()
            w = self.dist.all_to_all_single(o, i, group=self.group, async_op=async_op)
            if async_op:
                return _StagedWork(w, lambda: o, out)
            out.copy_(o)
            return None
        return self.dist.all_to_all_single(out, inp, group=self.group, async_op=async_op)

    def all_gather(self, out, inp, async_op=False, name="all_gather"):
        """out[s] = inp of rank s (dim 0 of out = ranks, inp flat or not)."""
        assert out.shape[0] == self.world and out.numel() == self.world * inp.numel()
        assert out.is_contiguous() and inp.is_contiguous()
        if self.world == 1 and not self.loop:
            if out.data_ptr() != inp.data_ptr():
                out.view(-1).copy_(inp.reshape(-1))
            return None
        # every other rank receives this rank's chunk
        self._count(name, inp.numel() * inp.element_size() * (self.world - 1))
        if self.staged and out.is_cuda:
            parts = [torch.empty(inp.shape, dtype=inp.dtype) for _ in range(self.world)]
            w = self.dist.all_gather(parts, inp.cpu(), group=self.group, async_op=async_op)

            def host():
                return torch.stack([p.reshape(-1) for p in parts]).view(out.shape)
            if async_op:
                return _StagedWork(w, host, out)
            out.copy_(host())
            return None
        return self.dist.all_gather_into_tensor(out.view(-1), inp.view(-1), group=self.group,
                                                async_op=async_op)


class SoloExchange:
    """The exchange of a one-rank run (no process group): ShardedBroadcast
    aliases its buffers, so nothing moves."""

    world, rank, staged, backend = 1, 0, True, "none"
    stats = {}

    def all_to_all(self, out, inp, async_op=False, name=None):
        if out.data_ptr() != inp.data_ptr():
            out.copy_(inp)

    def all_gather(self, out, inp, async_op=False, name=None):
        if out.data_ptr() != inp.data_ptr():
            out.view(-1).copy_(inp.reshape(-1))

    def reset_stats(self):
        pass


class CommTimer:
    """Collectives issued from a side stream, bracketed by timing events there.
    The side stream first waits for the data (an event recorded on the
    compute stream), so start -> end is the time the exchange occupies, also
    when it overlaps compute of other sub-batches.  run() returns the event
    the compute stream waits on before it reads the exchanged buffers."""

    def __init__(self, device):
        self.cs = torch.cuda.Stream(device)
        self.spans = []
        self.timing = False

    def run(self, fn):
        ready = torch.cuda.Event()
        ready.record()
        self.cs.wait_event(ready)
        with torch.cuda.stream(self.cs):
            a = torch.cuda.Event(enable_timing=True) if self.timing else None
            if a is not None:
                a.record()
            for h in fn():
                if h is not None:
                    h.wait()
            b = torch.cuda.Event(enable_timing=self.timing)
            b.record()
        if a is not None:
            self.spans.append((a, b))
        return b

    def elapsed_ms(self):
        return sum(a.elapsed_time(b) for a, b in self.spans)

    def reset(self):
        self.spans = []


# --------------------------------------------------------------- one rank ---
class ShardedBroadcast:
    """The per-rank state of the validator-sharded simulation: `count` local
    proposals of `plen` bytes per step on `device`."""

    def __init__(self, n, count, plen, rank, world, device=0, specialise=True, sm_slots=1):
        self.topo = t = Topology(n, world)
        self.rank, self.world, self.count, self.plen = rank, world, count, plen
        self.rb = rb = RbcBatch(n, t.f, device=device)
        dev = rb.device
        self.device = dev
        self.S = S = shard_len(plen, rb.k)
        self.stride = stride = rb.stride_for(S)
        self.ds = ds = max(rb.dslots, 1)
        self.dsz = ds * 32 + 16                 # digests ++ ndig ++ pad per row
        G, R, C = world, t.rpg, count
        self.rpb = t.rows_per_block
        u8 = dict(dtype=torch.uint8, device=dev)
        self.proposers = t.proposers(rank, C)
        # proposer side: destination-major slab [G][C][R][stride] (plain [C][n] at G=1)
        self.slab = torch.zeros((G, C, R, stride), **u8)
        self.nodes = rb.alloc_nodes(C)
        self.digests = torch.zeros((C, n, ds, 32), **u8)
        self.ndig = torch.zeros((C, n), **u8)
        # Value exchange
        self.dg_flat = torch.zeros((C, t.npad, self.dsz), **u8)
        self.send_dg = torch.zeros((G, C, R, self.dsz), **u8)
        self.recv_sh = self.slab if G == 1 else torch.empty_like(self.slab)
        self.recv_dg = self.send_dg if G == 1 else torch.empty_like(self.send_dg)
        self.roots_all = torch.empty((G, C, 32), **u8)
        # validator side: Value proofs of this rank's rows of every instance
        self.vreal = len(t.validators(rank))
        self.vrows_t = torch.arange(self.vreal, dtype=torch.int32, device=dev)
        idx = torch.arange(rank * R, rank * R + self.vreal, dtype=torch.int32, device=dev)
        self.recv_idx = idx.view(1, self.vreal).expand(G * C, self.vreal).contiguous()
        self.ok_v = torch.zeros((G * C, self.vreal), **u8)
        # every validator's Value outcome (= whether it sends Echo/EchoHash),
        # all-gathered with the Echoes: the Ready quorum counts them all
        self.ok_pad = torch.zeros((G * C, R), **u8)
        self.okv_all = self.ok_pad.view(1, G * C, R) if G == 1 else torch.zeros((G, G * C, R), **u8)
        self.v_digests = torch.zeros((G * C, R, ds, 32), **u8)
        self.v_ndig = torch.zeros((G * C, R), **u8)
        # Echo all-gather: every row of every instance, [G_v][G*C][R][stride]
        self.echo_sh = self.recv_sh if G == 1 else torch.empty((G, G * C, R, stride), **u8)
        self.echo_dg = self.recv_dg if G == 1 else torch.empty((G, G * C, R, self.dsz), **u8)
        self.e_digests = self.digests if G == 1 else torch.zeros((G * C, t.npad, ds, 32), **u8)
        self.e_ndig = self.ndig if G == 1 else torch.zeros((G * C, t.npad), **u8)
        self.echo_rows = t.echo_rows(rank) if G > 1 else []
        self.echo_rows_t = torch.tensor(self.echo_rows or [0], dtype=torch.int32, device=dev)
        self.ok_e = torch.zeros((G * C, max(1, len(self.echo_rows))), **u8)
        # receiver side: decode of every instance of every rank
        pres = t.receiver_present(rank)
        self.pattern = pres
        own = [j for j in t.validators(rank) if pres[j]]
        self.own_present = own
        self.present = torch.zeros((G * C, n), **u8)
        self.dec_nodes = rb.alloc_nodes(G * C)
        self.out = torch.zeros((G * C, max(16, (rb.k * S + 15) // 16 * 16)), **u8)
        self.plen_out = torch.zeros(G * C, dtype=torch.int32, device=dev)
        self.status = torch.zeros(G * C, dtype=torch.int32, device=dev)
        # RBC thresholds per instance (GPU-resident counters)
        self.echo_senders = torch.zeros(G * C, dtype=torch.int32, device=dev)
        self.full_echos = torch.zeros(G * C, dtype=torch.int32, device=dev)
        self.decided = torch.zeros(G * C, dtype=torch.bool, device=dev)
        # the Broadcast state machine of every hosted validator for every
        # instance (hbbft_amd/rbc_sim.py, sim.hip): Echo / EchoHash / Ready /
        # CanDecode handling with per-node counters, fed by this step's
        # validations and decodes; instance (s, i) = s * C + i, proposed by
        # validator proposers(s, C)[i]
        from .rbc_sim import StateMachineRank, honest_tensors
        props = [p_ for s_ in range(G) for p_ in t.proposers(s_, C)]
        # sm_slots = 2: two state machines with their own outcome buffers, so
        # the rounds of step i (a side stream) can run while step i + 1's data
        # plane fills the other slot's outcomes (overlapped_steps)
        sc = honest_tensors(n, props, dev)
        self.sms = []
        for _ in range(sm_slots):
            ok = torch.zeros((G * C, 1, 2, n), dtype=torch.uint8, device=dev)
            dec = torch.zeros((G * C, 1), dtype=torch.uint8, device=dev)
            self.sms.append(StateMachineRank(n, G * C, 1, sc, rank, world, device=device,
                                             max_out=4, max_faults=4, ok=ok, dec=dec))
        self.slot = 0
        self.sm_rounds = 0
        self.sm_timing = None   # a list: (start, end) events of every run_state_machines
        self.own_cols = torch.tensor([j - rank * R for j in own] or [0], dtype=torch.int64,
                                     device=dev)
        self.own_rows = torch.tensor(own or [0], dtype=torch.int64, device=dev)
        self.echo_cols = torch.tensor(self.echo_rows or [0], dtype=torch.int64, device=dev)
        rb.reserve(G * C)
        if specialise:
            rb.specialise_decoder(pres, self.rpb)

    # layouts: (shard_stride, rows_per_block, block_stride, inst_stride) --------
    def _prop_layout(self):
        G, R, C, st = self.world, self.topo.rpg, self.count, self.stride
        if G == 1:
            return st, 0, 0, self.topo.n * st
        return st, R, C * R * st, R * st

    def _echo_layout(self):
        G, R, C, st = self.world, self.topo.rpg, self.count, self.stride
        if G == 1:
            return st, 0, 0, self.topo.n * st
        return st, R, G * C * R * st, R * st

    # 1. proposer: frame, encode, tree, proofs -------------------------------
    def propose(self, payloads):
        rb, S, C, n = self.rb, self.S, self.count, self.topo.n
        st, rpb, bst, ist = self._prop_layout()
        rb.frame_encode_rows(payloads, self.plen, self.slab, C, st, rpb, bst, ist)
        rb.merkle_rows(self.slab, S, C, st, rpb, bst, ist, self.nodes)
        rb.proofs(self.nodes, self.digests, self.ndig)

    def roots(self):
        return self.nodes[:, -1, :]

    # 2. Value messages ---------------------------------------------------------
    def pack_value(self):
        """Digests (+ their counts) regrouped destination-major next to the
        slab, which the encoder already wrote that way (metadata only)."""
        if self.world == 1:
            return
        G, R, C, ds, n = self.world, self.topo.rpg, self.count, self.ds, self.topo.n
        self.dg_flat[:, :n, : ds * 32].copy_(self.digests.view(C, n, ds * 32))
        self.dg_flat[:, :n, ds * 32].copy_(self.ndig)
        self.send_dg.copy_(self.dg_flat.view(C, G, R, self.dsz).transpose(0, 1))

    def exchange_value(self, ex, async_op=False):
        """Value messages (+ the roots' all-gather); returns the handles."""
        self._roots = self.roots().contiguous()   # kept alive while in flight
        if self.world == 1:
            self.roots_all[0].copy_(self._roots)
            return []
        return [ex.all_to_all(self.recv_sh, self.slab, async_op, name="value_shards"),
                ex.all_to_all(self.recv_dg, self.send_dg, async_op, name="value_proofs"),
                ex.all_gather(self.roots_all, self._roots, async_op, name="roots")]

    # 3. validators validate their Values --------------------------------------
    def validate_values(self):
        G, R, C, ds, n = self.world, self.topo.rpg, self.count, self.ds, self.topo.n
        if G == 1:
            dig, nd, drows, ist = self.digests, self.ndig, n, n * self.stride
        else:
            src = self.recv_dg.view(G * C, R, self.dsz)
            self.v_digests.view(G * C, R, ds * 32).copy_(src[..., : ds * 32])
            self.v_ndig.copy_(src[..., ds * 32])
            dig, nd, drows, ist = self.v_digests, self.v_ndig, R, R * self.stride
        # this rank's rows of every instance, [G*C][R][stride]; their leaves go
        # to level 0 of the decode trees at index rank*R + r
        self.rb.validate_layout(self.recv_sh, self.S, G * C, self.vreal, self.stride, 0, 0, ist,
                                dig, nd, drows, self.roots_all.view(G * C, 32), self.ok_v,
                                rows=self.vrows_t, indices=self.recv_idx,
                                leaf_out=self.dec_nodes[:, self.rank * R:])
        self.ok_pad[:, : self.vreal].copy_(self.ok_v)

    # 4. Echo messages: all-gather of the validated rows ------------------------
    def exchange_echo(self, ex, async_op=False):
        if self.world == 1:
            return []
        return [ex.all_gather(self.echo_sh, self.recv_sh, async_op, name="echo_shards"),
                ex.all_gather(self.echo_dg, self.recv_dg, async_op, name="echo_proofs"),
                ex.all_gather(self.okv_all, self.ok_pad, async_op, name="echo_value_ok")]

    def validate_echoes(self):
        """Proof::validate of every Echo the receiver gets from other ranks'
        validators (handle_echo, broadcast.rs:291); the leaves go to the
        decode trees."""
        G, R, C, ds = self.world, self.topo.rpg, self.count, self.ds
        if G == 1 or not self.echo_rows:
            return
        # digests of every row of every instance in the validate layout [G*C][npad]
        src = self.echo_dg.view(G, G * C, R, self.dsz)
        self.e_digests.view(G * C, G, R, ds * 32).copy_(src[..., : ds * 32].transpose(0, 1))
        self.e_ndig.view(G * C, G, R).copy_(src[..., ds * 32].transpose(0, 1))
        st, rpb, bst, ist = self._echo_layout()
        self.rb.validate_layout(self.echo_sh, self.S, G * C, len(self.echo_rows), st, rpb, bst,
                                ist, self.e_digests, self.e_ndig, self.topo.npad,
                                self.roots_all.view(G * C, 32), self.ok_e,
                                rows=self.echo_rows_t, leaf_out=self.dec_nodes)

    # 5. every rank decodes every instance ------------------------------------
    def decode(self):
        self.present.zero_()
        if self.own_present:
            self.present[:, self.own_rows] = self.ok_v[:, self.own_cols]
        if self.echo_rows:
            self.present[:, self.echo_cols] = self.ok_e[:, : len(self.echo_rows)]
        st, rpb, bst, ist = self._echo_layout()
        self.rb.decode_rows(self.echo_sh, self.S, self.world * self.count, st, rpb, bst, ist,
                            self.present, self.roots_all.view(-1, 32), self.dec_nodes, self.out,
                            self.plen_out, self.status, known_leaves=True)
        self.thresholds()

    @property
    def sm(self):
        """The state machine of the current slot."""
        return self.sms[self.slot]

    def thresholds(self):
        """Inputs of the state machine from this step's data plane: proof (0,
        j) of every instance validates iff validator j's Value did (the Echo
        it forwards is the same proof, broadcast.rs:254, 291), and root 0
        decodes iff this rank's decode of the instance succeeded (a codeword
        decodes from any k of its rows, 551-557); plus the data-plane counts
        echo_senders (validators whose Value validated, i.e. that send Echo /
        EchoHash, 413-425, 456-468) and full_echos (Echoes receiver r0 holds)."""
        t, G, C = self.topo, self.world, self.count
        valid = self.okv_all.transpose(0, 1).reshape(G * C, t.npad)[:, : t.n]
        torch.sum(valid, dim=1, dtype=torch.int32, out=self.echo_senders)
        torch.sum(self.present, dim=1, dtype=torch.int32, out=self.full_echos)
        self.sm.ok[:, 0, 0, :].copy_(valid)
        self.sm.dec[:, 0].copy_(self.status == 0)

    def finish(self):
        """After the state machine's rounds: decided[i] = every validator this
        rank hosts output instance i (compute_output, broadcast.rs:526-558:
        > 2f Readys and >= k full Echoes, Ready sent at N - f Echoes or f + 1
        Readys)."""
        out = self.sm.output_root[:, : self.vreal]
        torch.all(out == 0, dim=1, out=self.decided)

    def state_machine(self, ex):
        self.sm_rounds = run_state_machines([self], ex)

    def encode_phase(self, payloads):
        """The proposer's frame + encode (the first kernel of a step)."""
        rb, C = self.rb, self.count
        st, rpb, bst, ist = self._prop_layout()
        rb.frame_encode_rows(payloads, self.plen, self.slab, C, st, rpb, bst, ist)

    def rest_phase(self, ex, xspans=None):
        """Everything of a step after the encoder: tree, proofs, exchanges,
        validation, decode (which leaves the state machine's outcomes in the
        current slot).  xspans: a list receiving (start, end) timing events
        around each exchange on the current stream (world > 1)."""
        rb, S, C = self.rb, self.S, self.count
        st, rpb, bst, ist = self._prop_layout()
        rb.merkle_rows(self.slab, S, C, st, rpb, bst, ist, self.nodes)
        rb.proofs(self.nodes, self.digests, self.ndig)
        self.pack_value()
        _timed(xspans, self.world, lambda: self.exchange_value(ex))
        self.validate_values()
        _timed(xspans, self.world, lambda: self.exchange_echo(ex))
        self.validate_echoes()
        self.decode()

    def data_step(self, payloads, ex):
        """Propose, exchange, validate and decode (the data plane of a step);
        the decode leaves the state machine's outcomes in the current slot."""
        self.propose(payloads)
        self.pack_value()
        self.exchange_value(ex)
        self.validate_values()
        self.exchange_echo(ex)
        self.validate_echoes()
        self.decode()

    def step(self, payloads, ex):
        self.data_step(payloads, ex)
        self.state_machine(ex)

    # accounting --------------------------------------------------------------
    def counts(self):
        """Per-step work of this rank: executed (per-GPU dedup) and faithful
        (every receiver of this rank's block, as the reference runs them)."""
        t, inst = self.topo, self.world * self.count
        present = sum(self.pattern)
        return {
            "value_validates": inst * self.vreal,
            "echo_validates": inst * len(self.echo_rows),
            "decodes": inst,
            "decode_leaf_hashes": inst * (t.n - present),
            "faithful_value_validates": inst * self.vreal,
            "faithful_echo_validates": inst * self.vreal * (t.n - t.f),
            "faithful_decodes": inst * self.vreal,
            "faithful_decode_leaf_hashes": inst * self.vreal * t.n,
            "state_machine_nodes": inst * self.vreal,
            "state_machine_rounds": self.sm_rounds,
            "state_machine_messages": self.sm.records,
        }


def _timed(spans, world, fn):
    """fn() between two timing events on the current stream when spans is a
    list and the exchange moves data (world > 1)."""
    if spans is None or world == 1:
        return fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    r = fn()
    b.record()
    spans.append((a, b))
    return r


HBM_PER_GPU = 288 * 10**9   # MI355X HBM3E


def rank_footprint(n, count, plen, world, rank=0, max_out=4, max_faults=4, sm_slots=1):
    """Device bytes one rank's ShardedBroadcast(n, count, plen, rank, world)
    allocates, by buffer, without a GPU: the torch tensors of __init__ (and
    of its StateMachineRank) at their exact shapes, aliases at world 1
    counted once, plus an upper bound of the library's reconstruct workspace
    (hbrbc_reserve: decode-matrix cache of cap + count slots, coefficient
    rows at one row per pass).  tests/test_sharded.py checks the torch part
    against torch.cuda.memory_allocated on the GPU."""
    from . import max_proof_len, merkle_node_count
    t = Topology(n, world)
    f = t.f
    k = n - 2 * f
    S = shard_len(plen, k)
    stride = (S + 15) // 16 * 16
    ds = max(max_proof_len(n), 1)
    dsz = ds * 32 + 16
    G, R, C = world, t.rpg, count
    nc = merkle_node_count(n)
    vreal = len(t.validators(rank))
    echo = t.echo_rows(rank) if G > 1 else []
    own = [j for j in t.validators(rank) if t.receiver_present(rank)[j]]
    W = (n + 31) // 32
    sm_state = _sm_state_bytes(n, 1)
    b = {
        "slab": G * C * R * stride,
        "nodes": C * nc * 32,
        "digests": C * n * ds * 32,
        "ndig": C * n,
        "dg_flat": C * t.npad * dsz,
        "send_dg": G * C * R * dsz,
        "roots_all": G * C * 32,
        "vrows_t": vreal * 4,
        "recv_idx": G * C * vreal * 4,
        "ok_v": G * C * vreal,
        "ok_pad": G * C * R,
        "v_digests": G * C * R * ds * 32,
        "v_ndig": G * C * R,
        "echo_rows_t": max(1, len(echo)) * 4,
        "ok_e": G * C * max(1, len(echo)),
        "present": G * C * n,
        "dec_nodes": G * C * nc * 32,
        "out": G * C * max(16, (k * S + 15) // 16 * 16),
        "plen_out": G * C * 4,
        "status": G * C * 4,
        "echo_senders": G * C * 4,
        "full_echos": G * C * 4,
        "decided": G * C,
        "sm_ok": sm_slots * G * C * 2 * n,
        "sm_dec": sm_slots * G * C,
        "own_cols": max(1, len(own)) * 8,
        "own_rows": max(1, len(own)) * 8,
        "echo_cols": max(1, len(echo)) * 8,
        # StateMachineRank (rbc_sim.py) of G * C instances, honest scenario
        # (honest_tensors: role / value_root / value_tamper share one [cnt][n])
        "sm_scenario": G * C * (1 + n + 2) + G * C * W * 4,
        "sm_state": sm_slots * (G * C * R * sm_state),
        "sm_out": sm_slots * (G * C * R * max_out * (1 + W) * 4),
        "sm_out_count": sm_slots * (G * C * R * 4),
        "sm_output_root": sm_slots * (G * C * R),
        "sm_faults": sm_slots * (G * C * R * max(1, max_faults) * 2),
        "sm_fault_count": sm_slots * (G * C * R * 4),
        "sm_hist": sm_slots * (64 * 2 * 4),          # per round: records, overflow (max_rounds 64)
        "sm_inbox": sm_slots * (G * G * C * R * max_out * (1 + W) * 4),
        "sm_inbox_count": sm_slots * (G * G * C * R * 4),
    }
    if G > 1:
        b.update({"recv_sh": G * C * R * stride, "recv_dg": G * C * R * dsz,
                  "okv_all": G * G * C * R, "echo_sh": G * G * C * R * stride,
                  "echo_dg": G * G * C * R * dsz, "e_digests": G * C * t.npad * ds * 32,
                  "e_ndig": G * C * t.npad})
    inst = G * C
    cap = 1024
    while cap < 2 * inst:
        cap *= 2
    slots = cap + inst
    lib_ws = (cap * 8 + slots * (32 + (2 * f * k * 16 + 16) + 4 * (k + 2 * f) + 8)
              + inst * (4 + 1 + 4) + (inst * max(2 * f, 1) + 1) * 8)
    torch_bytes = sum(b.values())
    return {"buffers": b, "torch_bytes": torch_bytes, "library_workspace_bound": lib_ws,
            "total_bytes": torch_bytes + lib_ws, "hbm_bytes": HBM_PER_GPU,
            "frac_of_hbm": (torch_bytes + lib_ws) / HBM_PER_GPU}


def _sm_state_bytes(n, roots):
    """hbrbc_sm_state_bytes (include/hbrbc.h) without loading the library:
    the per-node state block of sim.hip, 8-byte aligned."""
    from .rbc_sim import sm_state_bytes_host
    return sm_state_bytes_host(n, roots)


def pipelined_step(subs, payloads, ex, timer):
    """One step over several sub-batches (ShardedBroadcast objects on the same
    rank, payloads[i] for subs[i]) with every exchange in flight on the
    timer's side stream while the compute stream works on other sub-batches:
    propose all -> (Value of i overlaps propose of i+1) -> validate i while
    Value i+1 / Echo i-1 move -> decode i while Echo i+1 moves."""
    n = len(subs)
    ev_v, ev_e = [None] * n, [None] * n
    cur = torch.cuda.current_stream()
    for i, sb in enumerate(subs):
        sb.propose(payloads[i])
        sb.pack_value()
        ev_v[i] = timer.run(lambda sb=sb: sb.exchange_value(ex, async_op=True))
    for i, sb in enumerate(subs):
        cur.wait_event(ev_v[i])
        sb.validate_values()
        ev_e[i] = timer.run(lambda sb=sb: sb.exchange_echo(ex, async_op=True))
    for i, sb in enumerate(subs):
        cur.wait_event(ev_e[i])
        sb.validate_echoes()
        sb.decode()
    # every sub-batch's state machine in lockstep: one exchange per round
    rounds = run_state_machines(subs, ex)
    for sb in subs:
        sb.sm_rounds = rounds


class OverlapPipe:
    """The steps of one rank, the state machine of step i on the `side`
    stream beside the data plane of step i + 1 on the `main` stream (sb
    built with sm_slots=2; the slots alternate).  The rounds are
    latency-bound at low occupancy, the data plane's sponges issue-bound:
    side by side the GPU fills the one's idle issue slots with the other's
    work.  Step i's rounds start after step i + 1's encoder: the LDS-staged
    encoder needs 48 KB of LDS per workgroup and ran at half speed beside the
    rounds' LDS images (validator cfg4: encode 0.69 -> 1.50 ms), the sponge
    kernels use none.  `timing`: a list that receives (start, end) events of
    each step's rounds on the side stream.

    world > 1 (ex a DistExchange): the data plane's Value all-to-all and Echo
    all-gather run on `main` over `ex`; the rounds' per-round all-gathers
    (rbc_sim.DistRounds) run on `side` over `sm_ex`, which must hold a
    process group of its own (dist.new_group: its own RCCL communicator),
    so the two streams' collectives never interleave in a different order
    on different ranks.  Every rank enqueues the same collectives in the
    same order on each group, and a step's host read-back of the rounds of
    the step before waits only after this step's data plane is enqueued on
    every rank, so no rank can block a collective another rank waits for."""

    def __init__(self, sb, ex, side, main=None, timing=None, sm_ex=None, xspans=None):
        assert len(sb.sms) == 2
        if ex.world > 1 and (sm_ex is None or getattr(sm_ex, "group", None) is None
                             or sm_ex.group is getattr(ex, "group", None)):
            raise ValueError("world > 1: the overlapped state machine needs its own process "
                             "group (sm_ex = DistExchange(dist.new_group()))")
        self.sb, self.ex, self.side = sb, ex, side
        self.sm_ex = sm_ex if sm_ex is not None else ex
        self.main = main if main is not None else torch.cuda.current_stream()
        # the buffers and payloads were written on the caller's stream
        self.main.wait_stream(torch.cuda.current_stream())
        side.wait_stream(torch.cuda.current_stream())
        self.timing = timing
        self.xspans = xspans
        self.steps = 0
        self.prev_ready = None   # step i - 1's data plane is done (its outcomes are in)

    def _launch(self, slot, ready, after):
        from .rbc_sim import DistRounds, LocalRounds
        side = self.side
        side.wait_event(ready)
        if after is not None:
            side.wait_event(after)
        ev = None
        if self.timing is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(side)
            self.timing.append(ev)
        sms = [self.sb.sms[slot]]
        if self.sm_ex.world > 1:
            rounds = DistRounds(sms, self.sm_ex, stream=side).launch()
        else:   # one rank: its nodes only talk to themselves
            rounds = LocalRounds(sms, loopback=False, stream=side).launch()
        return slot, rounds, ev

    def _drain(self, p):
        slot, lr, ev = p
        sb = self.sb
        rounds = lr.wait()
        prev = sb.slot
        sb.slot = slot
        with torch.cuda.stream(self.side):
            sb.finish()
            if ev is not None:
                ev[1].record()
        sb.slot = prev
        sb.sm_rounds = rounds

    def step(self, payloads):
        """Enqueue one step; returns after the previous step's rounds."""
        sb, i = self.sb, self.steps
        with torch.cuda.stream(self.main):
            sb.slot = i % 2
            sb.encode_phase(payloads)
            after_encode = torch.cuda.Event()
            after_encode.record(self.main)
            running = None
            if self.prev_ready is not None:   # step i - 1's rounds, after step i's encoder
                running = self._launch((i - 1) % 2, self.prev_ready, after_encode)
            sb.rest_phase(self.ex, self.xspans)
            self.prev_ready = torch.cuda.Event()
            self.prev_ready.record(self.main)
        if running is not None:
            self._drain(running)              # host read; step i's data plane is queued
        self.steps += 1

    def finish(self):
        """Run the last step's rounds; every step's rounds have completed (and
        sb.decided holds the last step's flags) when this returns, and the
        caller's current stream waits for both streams."""
        if self.prev_ready is not None:
            self._drain(self._launch((self.steps - 1) % 2, self.prev_ready, None))
            self.prev_ready = None
        self.sb.slot = (self.steps - 1) % 2
        cur = torch.cuda.current_stream()
        cur.wait_stream(self.main)
        cur.wait_stream(self.side)


def overlapped_steps(sb, payloads, ex, steps, side, timing=None, sm_ex=None):
    """`steps` steps of one OverlapPipe on the current stream."""
    pipe = OverlapPipe(sb, ex, side, timing=timing, sm_ex=sm_ex)
    for _ in range(steps):
        pipe.step(payloads)
    pipe.finish()


def interleaved_steps(pipes, payloads, steps):
    """`steps` steps over several OverlapPipes on their own streams, step i
    on pipes[i % len(pipes)] (at world > 1 every rank steps the pipes in the
    same order, so each group's collectives keep one order across ranks):
    the pipes' data planes run side by side,
    so a sponge launch of one (4,096 lockstep waves at validator cfg3, one
    residency round) shares the SIMDs with another pipe's kernels instead of
    running in one synchronous round, and one pipe's rebuilt-row list and
    state machine leave their idle issue slots to the other."""
    for i in range(steps):
        pipes[i % len(pipes)].step(payloads[i % len(pipes)])
    for p in pipes:
        p.finish()


def run_state_machines(subs, ex):
    """Rounds of the Broadcast state machine (rbc_sim.run_rounds) of several
    ShardedBroadcast objects of this rank, their messages all-gathered over
    `ex` each round; then every object's decided flags."""
    from .rbc_sim import run_rounds
    ev = None
    if subs[0].sm_timing is not None:   # events around all rounds (host gaps included)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    if ex.world > 1:
        rounds = run_rounds([sb.sm for sb in subs], ex)
    else:   # one rank: each object's nodes only talk to themselves
        rounds = max(run_rounds([sb.sm]) for sb in subs)
    for sb in subs:
        sb.finish()
    if ev is not None:
        ev[1].record()
        subs[0].sm_timing.append(ev)
    return rounds
