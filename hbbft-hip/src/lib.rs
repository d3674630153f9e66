//! hbbft-hip: the MI355X backend of hbbft's Reliable-Broadcast data path.
//!
//! hbbft routes its data work through three private items -- `enum Coding`
//! (src/broadcast/broadcast.rs:639-694), `MerkleTree` (merkle.rs:12-69) and
//! `Proof` (merkle.rs:72-124).  This crate is what their bodies delegate to
//!: the same signatures and outcomes, every
//! computation in libhbrbc.so (HIP kernels for gfx950).  `ffi` is the whole C
//! ABI of include/hbrbc.h, generated from the header by gen_ffi.py; the batched
//! entry points (thousands of instances per call, device buffers, a
//! hipStream_t) are used through it directly.
//!
//! Not compiled in the image this was written in (no Rust toolchain there);
//! tests/test_crate.py checks ffi.rs against the header and the built library.
pub mod ffi;

use std::os::raw::c_int;

/// `reed_solomon_erasure::Error` for an hbrbc status 1..=13 (declaration
/// order).  Any other status is not an outcome rse could produce -- a HIP
/// failure (101), no visible GPU (102), a misuse of the ABI (100) -- and
/// panics with the library's message instead of posing as an rse error.
pub fn rse_error(code: c_int) -> reed_solomon_erasure::Error {
    use reed_solomon_erasure::Error::*;
    match code {
        1 => TooFewShards,
        2 => TooManyShards,
        3 => TooFewDataShards,
        4 => TooManyDataShards,
        5 => TooFewParityShards,
        6 => TooManyParityShards,
        7 => TooFewBufferShards,
        8 => TooManyBufferShards,
        9 => IncorrectShardSize,
        10 => TooFewShardsPresent,
        11 => EmptyShard,
        12 => InvalidShardFlags,
        13 => InvalidIndex,
        other => fail_loudly(other),
    }
}

/// A library or device failure: abort the caller with hbrbc_last_error().
pub fn fail_loudly(code: c_int) -> ! {
    let msg = unsafe { std::ffi::CStr::from_ptr(ffi::hbrbc_last_error()) };
    panic!("libhbrbc status {}: {}", code, msg.to_string_lossy());
}

type RseResult<T> = Result<T, reed_solomon_erasure::Error>;

/// `Coding` (broadcast.rs:639-694): one coding context per (data, parity),
/// parity 0 being the reference's `Coding::Trivial`.
#[derive(Debug)]
pub struct Coding(*mut ffi::HbrbcCtx);

// the context serialises its own host staging (a mutex inside the library)
unsafe impl Send for Coding {}
unsafe impl Sync for Coding {}

impl Drop for Coding {
    fn drop(&mut self) {
        unsafe { ffi::hbrbc_coding_free(self.0) }
    }
}

impl Coding {
    /// `Coding::new` (broadcast.rs:646-655; rse `ReedSolomon::new`).
    pub fn new(data_shard_num: usize, parity_shard_num: usize) -> RseResult<Self> {
        let mut ctx = std::ptr::null_mut();
        match unsafe { ffi::hbrbc_coding_new(data_shard_num, parity_shard_num, -1, &mut ctx) } {
            0 => Ok(Coding(ctx)),
            e => Err(rse_error(e)),
        }
    }

    pub fn data_shard_count(&self) -> usize {
        unsafe { ffi::hbrbc_data_shard_count(self.0) }
    }

    pub fn parity_shard_count(&self) -> usize {
        unsafe { ffi::hbrbc_parity_shard_count(self.0) }
    }

    /// `Coding::encode` (broadcast.rs:674-679): parity written in place.
    pub fn encode(&self, slices: &mut [&mut [u8]]) -> RseResult<()> {
        let ptrs: Vec<*mut u8> = slices.iter_mut().map(|s| s.as_mut_ptr()).collect();
        let lens: Vec<usize> = slices.iter().map(|s| s.len()).collect();
        match unsafe { ffi::hbrbc_encode(self.0, ptrs.as_ptr(), lens.as_ptr(), ptrs.len()) } {
            0 => Ok(()),
            e => Err(rse_error(e)),
        }
    }

    /// `Coding::reconstruct_shards` (broadcast.rs:682-693): missing shards
    /// are allocated zero-filled (as rse does) and rebuilt in place.
    pub fn reconstruct_shards(&self, shards: &mut [Option<Box<[u8]>>]) -> RseResult<()> {
        let len = shards.iter().flatten().map(|s| s.len()).next().unwrap_or(0);
        let present: Vec<u8> = shards.iter().map(|s| s.is_some() as u8).collect();
        let lens: Vec<usize> = shards.iter().map(|s| s.as_ref().map_or(0, |b| b.len())).collect();
        let mut bufs: Vec<Box<[u8]>> = shards
            .iter_mut()
            .map(|s| s.take().unwrap_or_else(|| vec![0u8; len].into_boxed_slice()))
            .collect();
        let ptrs: Vec<*mut u8> = bufs.iter_mut().map(|b| b.as_mut_ptr()).collect();
        let st = unsafe {
            ffi::hbrbc_reconstruct(self.0, ptrs.as_ptr(), lens.as_ptr(), present.as_ptr(), ptrs.len())
        };
        for (slot, (b, p)) in shards.iter_mut().zip(bufs.into_iter().zip(&present)) {
            if *p == 1 || st == 0 {
                *slot = Some(b); // on error the absent ones stay None
            }
        }
        match st {
            0 => Ok(()),
            e => Err(rse_error(e)),
        }
    }
}

/// The flattened node slab of `MerkleTree::from_vec` (merkle.rs:20-33): the
/// tree's `levels` (leaf digests first, the root's level excluded, as the
/// reference stores them) and its `root_hash`.
pub fn merkle_from_vec<T: AsRef<[u8]>>(values: &[T]) -> (Vec<Vec<[u8; 32]>>, [u8; 32]) {
    let n = values.len();
    let ptrs: Vec<*const u8> = values.iter().map(|v| v.as_ref().as_ptr()).collect();
    let lens: Vec<usize> = values.iter().map(|v| v.as_ref().len()).collect();
    let mut nodes = vec![[0u8; 32]; unsafe { ffi::hbrbc_merkle_node_count(n) }];
    let st = unsafe {
        ffi::hbrbc_merkle_build(ptrs.as_ptr(), lens.as_ptr(), n, nodes.as_mut_ptr() as *mut u8)
    };
    if st != 0 {
        fail_loudly(st) // the reference panics on n == 0 too
    }
    let mut levels = Vec::new();
    let (mut off, mut sz) = (0, n);
    while sz > 1 {
        levels.push(nodes[off..off + sz].to_vec());
        off += sz;
        sz = (sz + 1) / 2;
    }
    (levels, nodes[off])
}

/// `Proof::validate` (merkle.rs:83-103) of (value, index, digests, root) in a
/// tree over n leaves.  A device failure panics: it is not an invalid proof.
///
/// Per call this is slower than the CPU: 651 µs against 49 µs for
/// tiny-keccak on one core at N=64 with 11,916-byte shards, 359 / 29 µs at
/// N=128, 62 / 12 µs at N=4 (profiles/r3_percall_pair.jsonl).  One proof is a
/// serial chain of permutations.  Batch proofs through
/// `hbrbc_validate_batch` instead; use this only behind an opt-in feature.
pub fn proof_validate(value: &[u8], index: usize, digests: &[[u8; 32]], root: &[u8; 32], n: usize) -> bool {
    let mut ok: c_int = 0;
    let st = unsafe {
        ffi::hbrbc_proof_validate(value.as_ptr(), value.len(), index, digests.as_ptr() as *const u8,
                                  digests.len(), root.as_ptr(), n, &mut ok)
    };
    if st != 0 {
        fail_loudly(st)
    }
    ok == 1
}

/// `e(a, b) == e(c, d)` on the GPU (threshold_decrypt.rs:142, 220-228 through
/// threshold_crypto), points in the pairing crate's uncompressed encodings.
pub fn pairing_eq(a: &[u8; 96], b: &[u8; 192], c: &[u8; 96], d: &[u8; 192]) -> bool {
    let mut r: c_int = 0;
    let st = unsafe { ffi::hbrbc_pairing_check(a.as_ptr(), b.as_ptr(), c.as_ptr(), d.as_ptr(), &mut r) };
    if st != 0 {
        fail_loudly(st) // valid typed points never fail; a device error panics
    }
    r == 1
}
