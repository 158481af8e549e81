//! The stream writer's ordered encode stage (sdk/src/stream/write.rs:332-362: up to
//! min(cores, 4) chunk encodes in flight, handed on in order through FuturesOrdered) over
//! te_stream_writer: one GPU pipeline per ClayCoder (one per device), windows enqueued without
//! blocking, completed in submission order.  Each window is `encode_with_proofs` of its objects
//! (sdk/src/codec/encoder.rs:220-260).
use crate::{encode_status, pack_objects, slicer_cfg, ClayCoder, EncodeError, ErasureCoder, PinnedBuf, PinnedPool};
use std::collections::BTreeMap;
use tapeec_sys as ffi;

struct Pending { data: PinnedBuf, objs: Vec<ffi::te_object>, out: crate::EncodedWindow }

/// Who hashes the leaves (te_stream_writer_set_hashing): `Auto` picks per window -- the SDK's
/// 64 MiB chunks (9.7 MB slices, <= 4 in flight) hash on the library's host pool as their slices
/// land, batches of small objects on the device.
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub enum Hashing { Auto, Device, Host }

pub struct StreamWriter<'a> {
    raw: *mut ffi::te_stream_writer,
    coders: Vec<&'a mut ClayCoder>,  // the handles outlive the writer (borrowed)
    pending: BTreeMap<u64, Pending>,
    pool: PinnedPool,                 // pinned input / slice buffers, reused across windows
}

impl<'a> StreamWriter<'a> {
    /// group_bytes: hashing group per handle (0 = 8 GiB); height: SLICE_TREE_HEIGHT.
    pub fn new(coders: Vec<&'a mut ClayCoder>, group_bytes: usize) -> Self {
        let raws: Vec<*mut ffi::te_clay> = coders.iter().map(|c| c.raw.as_ptr()).collect();
        let cfg = slicer_cfg(&*coders[0], true, 0);
        let mut w = std::ptr::null_mut();
        let r = unsafe {
            ffi::te_stream_writer_new(raws.as_ptr(), raws.len(), &cfg, ffi::TE_SLICE_TREE_HEIGHT as u32, group_bytes, &mut w)
        };
        if r != 0 { crate::fatal(r) }
        Self { raw: w, coders, pending: BTreeMap::new(), pool: PinnedPool::default() }
    }

    pub fn set_hashing(&mut self, h: Hashing) {
        let mode = match h { Hashing::Auto => ffi::TE_HASH_AUTO, Hashing::Device => ffi::TE_HASH_DEVICE, Hashing::Host => ffi::TE_HASH_HOST };
        let r = unsafe { ffi::te_stream_writer_set_hashing(self.raw, mode as i32) };
        if r != 0 { crate::fatal(r) }
    }

    /// Hand a completed window's pinned slice buffer back for reuse (after the slices are stored).
    pub fn recycle(&mut self, w: crate::EncodedWindow) { self.pool.give(w.slices) }

    /// Enqueue one window; returns its ticket.  The window's buffers stay owned here (stable
    /// addresses for the asynchronous copies) until `next` hands them back.
    pub fn submit(&mut self, objects: &[&[u8]], chunk_index: &[u64]) -> Result<u64, EncodeError> {
        let (data, objs, out_len) = pack_objects(&*self.coders[0], &mut self.pool, objects, chunk_index);
        let n = self.coders[0].n();
        let h = ffi::TE_SLICE_TREE_HEIGHT as usize;
        let mut p = Pending { data, objs, out: crate::EncodedWindow {
            slices: self.pool.take(out_len as usize), leaf_hashes: vec![0; objects.len() * n * 32],
            roots: vec![0; objects.len() * 32], proofs: vec![0; objects.len() * n * h * 32] } };
        let mut t = 0u64;
        let r = unsafe {
            ffi::te_stream_submit(self.raw, p.data.as_ptr(), p.objs.as_ptr(), p.objs.len(), p.out.slices.as_mut_ptr(),
                                  p.out.leaf_hashes.as_mut_ptr(), p.out.roots.as_mut_ptr(), p.out.proofs.as_mut_ptr(), &mut t)
        };
        // a failed window keeps its ticket: `next` reports it in order (its buffers are no longer
        // referenced by the device once submit has returned)
        if t != 0 { self.pending.insert(t, p); }
        encode_status(r)?;
        Ok(t)
    }

    /// Windows submitted and not yet handed back by `next`.
    pub fn in_flight(&self) -> usize { self.pending.len() }

    /// The oldest window, completed (FuturesOrdered::next).
    pub fn next(&mut self) -> Option<Result<crate::EncodedWindow, EncodeError>> {
        let (&t, _) = self.pending.iter().next()?;
        let r = unsafe { ffi::te_stream_wait(self.raw, t) };
        let p = self.pending.remove(&t)?;
        self.pool.give(p.data);  // the window's input buffer is free once it has completed
        Some(encode_status(r).map(|_| p.out))
    }
}

impl Drop for StreamWriter<'_> {
    fn drop(&mut self) { unsafe { ffi::te_stream_writer_free(self.raw) } }
}
