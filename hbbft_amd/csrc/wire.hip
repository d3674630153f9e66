// wire.hip -- bincode wire format of broadcast::Message on the GPU.
//
// Reference: /root/reference/src/broadcast/message.rs:13-24 (`Message`),
// merkle.rs:72-78 (`Proof` field order: value, index, digests, root_hash),
// serialised with bincode 1.x defaults (`bincode = "1.2.0"`, Cargo.toml:24;
// `bincode::serialize` in examples/simulation.rs:132,185 and
// `serialize_into` in examples/network/commst.rs:68): little-endian, fixed
// width integers, enum variant as u32, sequence lengths and usize as u64,
// [u8; 32] as 32 raw bytes.  A Value / Echo message is
//
//   off 0          u32 variant (0 Value, 1 Echo; 2 Ready, 3 CanDecode, 4 EchoHash)
//   off 4          u64 L = value length
//   off 12         L value bytes
//   off 12+L       u64 index
//   off 20+L       u64 d = number of digests
//   off 28+L       d x 32 digest bytes
//   off 28+L+32d   32 root bytes                      total 60 + L + 32 d
//
// and a Ready / CanDecode / EchoHash message is the u32 variant + 32 bytes.
//
// Messages live in fixed slots of `msg_stride` bytes (16-aligned).  The value
// body -- nearly all the bytes -- moves as aligned 16-byte chunks with a
// compile-time register shift (the body starts 12 bytes into a 16-aligned
// slot); the headers, digests and roots are assembled byte by byte by the few
// lanes whose chunk touches them.
#include "device_common.hpp"
#include "launchers.hpp"

namespace hbrbc {

namespace {

constexpr int kWireBlock = 256;

// Byte b of a little-endian integer.
__device__ __forceinline__ uint32_t le_byte(uint64_t v, uint32_t b) {
    return (uint32_t)(v >> (8 * b)) & 0xFFu;
}

// One thread per 16-byte chunk of every message slot.
__global__ __launch_bounds__(kWireBlock) void wire_encode_kernel(
    uint32_t variant, const uint8_t *__restrict__ values, uint32_t L, size_t value_stride,
    size_t value_inst_stride, uint32_t per_inst, const uint32_t *__restrict__ indices,
    const uint8_t *__restrict__ digests, uint32_t dslots, const uint8_t *__restrict__ ndig,
    const uint8_t *__restrict__ roots, size_t root_stride, uint8_t *__restrict__ out,
    size_t msg_stride, uint32_t *__restrict__ msg_len, uint32_t chunks_per_slot,
    uint32_t blocks_per_msg) {
    const size_t msg = blockIdx.x / blocks_per_msg;  // scalar
    const uint32_t c = (uint32_t)(blockIdx.x - msg * blocks_per_msg) * kWireBlock + threadIdx.x;
    if (c >= chunks_per_slot) return;
    const size_t inst = msg / per_inst;
    const uint32_t j = (uint32_t)(msg - inst * per_inst);
    const uint32_t d = ndig[msg];
    const uint32_t total = 60u + L + 32u * d;
    if (c == 0) msg_len[msg] = total;
    const uint32_t o = c * 16u;
    uint8_t *dst = out + msg * msg_stride + o;
    if (o >= total) {
        *reinterpret_cast<uint4 *>(dst) = make_uint4(0, 0, 0, 0);  // slot padding
        return;
    }
    const uint8_t *val = values + inst * value_inst_stride + (size_t)j * value_stride;
    if (o >= 12u && o + 16u <= 12u + L) {
        // value body: bytes [o-12, o+4) of the 16-aligned row = bytes 4..19 of
        // the aligned window at o-16
        const uint4 a = *reinterpret_cast<const uint4 *>(val + (o - 16u));
        const uint4 b = *reinterpret_cast<const uint4 *>(val + o);
        *reinterpret_cast<uint4 *>(dst) = make_uint4(a.y, a.z, a.w, b.x);
        return;
    }
    const uint32_t index = indices ? indices[msg] : j;
    const uint8_t *dg = digests + msg * (size_t)dslots * 32;
    const uint8_t *rt = roots + inst * root_stride;
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t t = 0; t < 16; ++t) {
        const uint32_t b = o + t;
        uint32_t v = 0;
        if (b >= total) v = 0;
        else if (b < 4) v = le_byte(variant, b);
        else if (b < 12) v = le_byte(L, b - 4);
        else if (b < 12 + L) v = val[b - 12];
        else if (b < 20 + L) v = le_byte(index, b - 12 - L);
        else if (b < 28 + L) v = le_byte(d, b - 20 - L);
        else if (b < 28 + L + 32 * d) v = dg[b - 28 - L];
        else v = rt[b - 28 - L - 32 * d];
        w[t >> 2] |= v << (8 * (t & 3));
    }
    *reinterpret_cast<uint4 *>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
}

// bincode deserialisation of every message header: variant, lengths,
// index, digests, root; status per message.
__global__ __launch_bounds__(kWireBlock) void wire_parse_kernel(
    const uint8_t *__restrict__ msgs, size_t msg_stride, const uint32_t *__restrict__ msg_len,
    size_t nmsg, uint32_t value_cap, uint32_t *__restrict__ value_len_out,
    uint32_t *__restrict__ index_out, uint8_t *__restrict__ digests, uint32_t dslots,
    uint8_t *__restrict__ ndig_out, uint8_t *__restrict__ roots,
    uint32_t *__restrict__ variant_out, int32_t *__restrict__ status_out) {
    const size_t g = blockIdx.x * (size_t)kWireBlock + threadIdx.x;
    if (g >= nmsg) return;
    const uint8_t *m = msgs + g * msg_stride;
    const uint64_t avail = min((uint64_t)msg_len[g], (uint64_t)msg_stride);  // never past the slot
    auto rd = [&](uint64_t off, int nbytes) {
        uint64_t v = 0;
        for (int b = 0; b < nbytes; ++b) v |= (uint64_t)m[off + b] << (8 * b);
        return v;
    };
    int32_t st = 0;
    uint32_t variant = 0, L = 0, index = 0, d = 0;
    uint64_t root_off = 0;
    if (avail < 4) {
        st = 70;  // truncated (bincode UnexpectedEof)
    } else {
        variant = (uint32_t)rd(0, 4);
        if (variant > 4) {
            st = 71;  // unknown enum variant
        } else if (variant >= 2) {
            if (avail < 36) st = 70;
            root_off = 4;
        } else if (avail < 12) {
            st = 70;
        } else {
            const uint64_t l64 = rd(4, 8);
            if (l64 > avail) {
                st = 70;
            } else if (l64 > value_cap) {
                st = 72;  // does not fit the value slab of this batch
            } else {
                L = (uint32_t)l64;
                if (avail < 28ull + L) {
                    st = 70;
                } else {
                    const uint64_t i64 = rd(12 + L, 8);
                    const uint64_t d64 = rd(20 + L, 8);
                    index = i64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)i64;
                    if (d64 > dslots) {
                        st = 72;  // more digests than any tree of this N has levels
                    } else if (avail < 60ull + L + 32 * d64) {
                        st = 70;
                    } else {
                        d = (uint32_t)d64;
                        uint8_t *dg = digests + g * (size_t)dslots * 32;
                        for (uint32_t b = 0; b < 32 * d; ++b) dg[b] = m[28 + L + b];
                        root_off = 28ull + L + 32ull * d;
                    }
                }
            }
        }
    }
    if (st == 0)
        for (int b = 0; b < 32; ++b) roots[g * 32 + b] = m[root_off + b];
    variant_out[g] = variant;
    value_len_out[g] = st ? 0 : L;
    index_out[g] = index;
    ndig_out[g] = (uint8_t)d;
    status_out[g] = st;
}

// Value bodies of parsed Value/Echo messages into 16-aligned rows: value
// bytes [16v, 16v+16) = message bytes [12+16v, 28+16v) = bytes 12..27 of the
// aligned window at 16v.  Bytes past L are written 0.
__global__ __launch_bounds__(kWireBlock) void wire_value_kernel(
    const uint8_t *__restrict__ msgs, size_t msg_stride, const int32_t *__restrict__ status,
    const uint32_t *__restrict__ variant, const uint32_t *__restrict__ value_len,
    uint8_t *__restrict__ values, size_t value_stride, uint32_t chunks_per_row,
    uint32_t blocks_per_row) {
    const size_t g = blockIdx.x / blocks_per_row;  // scalar
    const uint32_t v = (uint32_t)(blockIdx.x - g * blocks_per_row) * kWireBlock + threadIdx.x;
    if (v >= chunks_per_row) return;
    uint4 *dst = reinterpret_cast<uint4 *>(values + g * value_stride + 16u * v);
    const uint32_t L = value_len[g];
    if (status[g] != 0 || variant[g] > 1 || 16u * v >= L) {
        *dst = make_uint4(0, 0, 0, 0);
        return;
    }
    const uint8_t *m = msgs + g * msg_stride + 16u * v;
    const uint4 a = *reinterpret_cast<const uint4 *>(m);
    const uint4 b = *reinterpret_cast<const uint4 *>(m + 16);
    uint32_t w[4] = {a.w, b.x, b.y, b.z};
    const uint32_t keep = L - 16u * v;  // bytes of this chunk inside the value
    if (keep < 16) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = (int)keep - 4 * q;
            if (k <= 0) w[q] = 0;
            else if (k < 4) w[q] &= 0xFFFFFFFFu >> (8 * (4 - k));
        }
    }
    *dst = make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace

hipError_t launch_wire_encode(const WireEncodeArgs &a, hipStream_t s) {
    const size_t nmsg = a.count * a.per_inst;
    if (nmsg == 0) return hipSuccess;
    const uint32_t cps = (uint32_t)(a.msg_stride / 16);
    const uint32_t bpm = (cps + kWireBlock - 1) / kWireBlock;
    if (nmsg * bpm > 0xFFFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wire_encode_kernel, dim3((unsigned)(nmsg * bpm)), dim3(kWireBlock), 0, s,
                       a.variant, a.values, (uint32_t)a.value_len, a.value_stride,
                       a.value_inst_stride, (uint32_t)a.per_inst, a.indices, a.digests,
                       (uint32_t)a.dslots, a.ndig, a.roots, a.root_stride, a.out, a.msg_stride,
                       a.msg_len, cps, bpm);
    return hipGetLastError();
}

hipError_t launch_wire_decode(const WireDecodeArgs &a, hipStream_t s) {
    if (a.nmsg == 0) return hipSuccess;
    hipLaunchKernelGGL(wire_parse_kernel, dim3((unsigned)((a.nmsg + kWireBlock - 1) / kWireBlock)),
                       dim3(kWireBlock), 0, s, a.msgs, a.msg_stride, a.msg_len, a.nmsg,
                       (uint32_t)a.value_cap, a.value_len, a.index, a.digests, (uint32_t)a.dslots,
                       a.ndig, a.roots, a.variant, a.status);
    const uint32_t cpr = (uint32_t)(a.value_stride / 16);
    if (cpr == 0) return hipGetLastError();
    const uint32_t bpr = (cpr + kWireBlock - 1) / kWireBlock;
    if (a.nmsg * bpr > 0xFFFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wire_value_kernel, dim3((unsigned)(a.nmsg * bpr)), dim3(kWireBlock), 0, s,
                       a.msgs, a.msg_stride, a.status, a.variant, a.value_len, a.values,
                       a.value_stride, cpr, bpr);
    return hipGetLastError();
}

}  // namespace hbrbc
