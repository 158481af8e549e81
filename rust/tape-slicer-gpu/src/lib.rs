//! The reference's `lib/slicer` coders over libtapeec, as INTEGRATION.md describes: a drop-in
//! `ClayCoder` (clay.rs:13-122), `OuterCoder` (outer.rs:19-197) and the batched write-path call
//! (`encode_with_proofs` per object, sdk/src/codec/encoder.rs:220-260).  The reference crate's
//! error enums are restated here with the same variants so this file compiles on its own; inside
//! lib/slicer the `crate::errors` types replace them.
//!
//! Not compiled in this repository's CI (no Rust toolchain in the build image); the FFI it calls
//! is the generated `tapeec-sys`, which tests/test_rust_binding.py keeps in step with the header.
use std::ptr::NonNull;
use tapeec_sys as ffi;

#[derive(Debug, PartialEq, Eq)]
pub enum EncodeError { TooMuchData, EmptyInput }
#[derive(Debug, PartialEq, Eq)]
pub enum DecodeError { NotEnoughSlices, TooMuchData, BadEncoding, InvalidLayout }

fn fatal(status: i32) -> ! {
    let msg = unsafe { std::ffi::CStr::from_ptr(ffi::te_strerror(status)) };
    let detail = unsafe { std::ffi::CStr::from_ptr(ffi::te_last_error_detail()) };
    panic!("libtapeec: {} ({})", msg.to_string_lossy(), detail.to_string_lossy())
}

/// ClayCoder (lib/slicer/src/clay.rs:13-122) with the GF(2^8) work on the GPU.
pub struct ClayCoder { raw: NonNull<ffi::te_clay>, pub k: usize, pub m: usize, pub d: usize }
// libtapeec serialises calls on one handle internally; the handle is bound to its device.
unsafe impl Send for ClayCoder {}

impl ClayCoder {
    pub fn new(n: usize, k: usize, d: usize) -> Self {
        assert!(n > k, "n must be > k"); // clay.rs:24-34
        assert!(k > 0, "k must be > 0");
        assert!(d >= k + 1, "d must be >= k + 1");
        assert!(d <= n - 1, "d must be <= n - 1");
        let mut p = std::ptr::null_mut();
        let r = unsafe { ffi::te_clay_new(n as u32, k as u32, d as u32, &mut p) };
        if r != 0 { fatal(r) }
        Self { raw: NonNull::new(p).unwrap(), k, m: n - k, d }
    }
    pub fn n(&self) -> usize { self.k + self.m }
    pub fn chunk_size_for(&self, len: usize) -> usize { unsafe { ffi::te_clay_chunk_size_for(self.raw.as_ptr(), len) } }

    pub fn encode(&mut self, data: &[u8]) -> Result<Vec<Vec<u8>>, EncodeError> {
        if data.is_empty() { return Err(EncodeError::EmptyInput) }
        let cs = self.chunk_size_for(data.len());
        let mut buf = vec![0u8; self.n() * cs];
        let mut got = 0usize;
        match unsafe { ffi::te_clay_encode(self.raw.as_ptr(), data.as_ptr(), data.len(), buf.as_mut_ptr(), buf.len(), &mut got) } {
            0 => Ok(buf.chunks(got).map(<[u8]>::to_vec).collect()),
            1 => Err(EncodeError::TooMuchData),
            2 => Err(EncodeError::EmptyInput),
            s => fatal(s),
        }
    }

    pub fn decode(&mut self, chunks: &[(usize, &[u8])]) -> Result<Vec<u8>, DecodeError> {
        if chunks.len() < self.k { return Err(DecodeError::NotEnoughSlices) }
        let cs = chunks[0].1.len();
        let mut ptrs = vec![std::ptr::null::<u8>(); self.n()];
        for (i, c) in chunks {
            if c.len() != cs || *i >= self.n() { return Err(DecodeError::InvalidLayout) }
            ptrs[*i] = c.as_ptr();
        }
        let mut out = vec![0u8; self.k * cs];
        match unsafe { ffi::te_clay_decode(self.raw.as_ptr(), ptrs.as_ptr(), cs, out.as_mut_ptr(), out.len()) } {
            0 => Ok(out),
            3 => Err(DecodeError::NotEnoughSlices),
            5 => Err(DecodeError::InvalidLayout),
            4 => Err(DecodeError::BadEncoding),
            s => fatal(s),
        }
    }
}
impl Drop for ClayCoder { fn drop(&mut self) { unsafe { ffi::te_clay_free(self.raw.as_ptr()) } } }

/// OuterCoder (lib/slicer/src/outer.rs:19-197): GF(2^16) RS over n chunks, any k reconstruct.
pub struct OuterCoder { k: usize, n: usize }

impl OuterCoder {
    pub fn new(k: usize, n: usize) -> Self {
        assert!(k > 0, "k must be > 0");
        assert!(k <= n, "k must be <= n");
        Self { k, n }
    }
    pub fn encode(&mut self, data: &[u8]) -> Result<Vec<Vec<u8>>, EncodeError> {
        let cb = unsafe { ffi::te_outer_chunk_bytes(self.k as u32, data.len()) };
        let mut out = vec![0u8; self.n * cb];
        let mut got = 0usize;
        match unsafe { ffi::te_outer_encode(self.k as u32, self.n as u32, data.as_ptr(), data.len(), out.as_mut_ptr(), out.len(), &mut got) } {
            0 => Ok(out.chunks(cb).map(<[u8]>::to_vec).collect()),
            1 => Err(EncodeError::TooMuchData),
            s => fatal(s),
        }
    }
    pub fn decode(&mut self, chunks: &[(usize, &[u8])]) -> Result<Vec<u8>, DecodeError> {
        if chunks.len() < self.k { return Err(DecodeError::NotEnoughSlices) }
        let cb = chunks[0].1.len();
        let mut ptrs = vec![std::ptr::null::<u8>(); self.n];
        for (i, c) in chunks {
            if c.len() != cb || *i >= self.n { return Err(DecodeError::InvalidLayout) }
            ptrs[*i] = c.as_ptr();
        }
        let mut out = vec![0u8; self.k * cb];
        match unsafe { ffi::te_outer_decode(self.k as u32, self.n as u32, ptrs.as_ptr(), cb, out.as_mut_ptr(), out.len()) } {
            0 => Ok(out),
            3 => Err(DecodeError::NotEnoughSlices),
            5 => Err(DecodeError::InvalidLayout),
            s => fatal(s),
        }
    }
}

/// One window of the stream writer (sdk/src/stream/write.rs:332-362): every object's 20 slices
/// plus `encode_with_proofs`' leaf hashes, root and proofs, in one call.  Host buffers should be
/// pinned (hipHostRegister) for full PCIe rate.
pub struct EncodedWindow { pub slices: Vec<u8>, pub leaf_hashes: Vec<u8>, pub roots: Vec<u8>, pub proofs: Vec<u8> }

pub fn encode_with_proofs_batch(coder: &mut ClayCoder, objects: &[&[u8]], window_bytes: usize)
        -> Result<EncodedWindow, EncodeError> {
    let n = coder.n();
    let cfg = ffi::te_slicer_cfg { rotated: 1, encoding: ffi::TE_ENCODING_CLAY, params: ffi::TE_CLAY_DEFAULT_PARAMS, chunk_index: 0 };
    let mut data = Vec::new();
    let mut objs = Vec::with_capacity(objects.len());
    let mut out_len = 0u64;
    for o in objects {
        let mut g = ffi::te_geometry { stripe_size: 0, num_stripes: 0, chunk_size: 0, sub_chunk_size: 0, slice_len: 0 };
        unsafe { ffi::te_slicer_geometry(coder.raw.as_ptr(), o.len(), &mut g) };
        objs.push(ffi::te_object { data_off: data.len() as u64, blob_len: o.len() as u64, out_off: out_len, chunk_index: 0 });
        data.extend_from_slice(o);
        out_len += n as u64 * g.slice_len;
    }
    let h = ffi::TE_SLICE_TREE_HEIGHT as usize;
    let mut w = EncodedWindow { slices: vec![0; out_len as usize], leaf_hashes: vec![0; objects.len() * n * 32],
                                roots: vec![0; objects.len() * 32], proofs: vec![0; objects.len() * n * h * 32] };
    match unsafe { ffi::te_encode_commit_batch_host(coder.raw.as_ptr(), &cfg, data.as_ptr(), objs.as_ptr(), objs.len(),
                   w.slices.as_mut_ptr(), h as u32, w.leaf_hashes.as_mut_ptr(), w.roots.as_mut_ptr(),
                   w.proofs.as_mut_ptr(), window_bytes) } {
        0 => Ok(w),
        1 => Err(EncodeError::TooMuchData),
        s => fatal(s),
    }
}
