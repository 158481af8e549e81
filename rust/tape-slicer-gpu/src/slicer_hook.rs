//! The `Slicer` whole-object hook of INTEGRATION.md §4: `Slicer<C>` (slicer.rs:124-132) is generic
//! over `ErasureCoder`, and `ClayCoder` can do a whole object -- striping, the re-encode of the
//! short last stripe, rotation and the 48-byte suffix (slicer.rs:237-296), the per-stripe decode
//! (slicer.rs:298-364) and the per-stripe repair (repair.rs:324-367) -- in one library call that
//! launches one kernel per object instead of one per stripe.  lib/slicer adds the defaulted
//! `ObjectCoder` methods to its trait and tries them first:
//!
//! ```ignore
//! // Slicer::encode, slicer.rs:237
//! if let Some(r) = self.coder.encode_object(&self.object_cfg(), data) { return r; }
//! // Slicer::decode, slicer.rs:298
//! if let Some(r) = self.coder.decode_object(&self.object_cfg(), slices) { return r; }
//! ```
//!
//! keeping the per-stripe loops for the other coders (`ReedSolomonCoder`).
use crate::{decode_status, encode_status, repair_status, ClayCoder, DecodeError, EncodeError, ErasureCoder,
            RepairError, SliceIndex};
use tapeec_sys as ffi;

/// The Slicer fields the object path needs (slicer.rs:124-132): mapping strategy, the profile
/// written to the metadata suffix, the ChunkNumber salt.
#[derive(Clone, Copy, Debug)]
pub struct ObjectCfg { pub rotated: bool, pub encoding: u64, pub params: u64, pub chunk_index: u64 }

impl ObjectCfg {
    fn ffi(&self) -> ffi::te_slicer_cfg {
        ffi::te_slicer_cfg { rotated: self.rotated as i32, encoding: self.encoding, params: self.params,
                             chunk_index: self.chunk_index }
    }
}

/// Defaulted hooks: `None` = the coder has no object path, the Slicer runs its stripe loop.
pub trait ObjectCoder: ErasureCoder {
    fn encode_object(&mut self, _cfg: &ObjectCfg, _data: &[u8]) -> Option<Result<Vec<Vec<u8>>, EncodeError>> { None }
    fn decode_object(&mut self, _cfg: &ObjectCfg, _slices: &[(usize, &[u8])]) -> Option<Result<Vec<u8>, DecodeError>> {
        None
    }
}

impl ObjectCoder for ClayCoder {
    /// Slicer::encode (slicer.rs:237-296 + encode_empty_blob :368-387) in one te_slicer_encode.
    fn encode_object(&mut self, cfg: &ObjectCfg, data: &[u8]) -> Option<Result<Vec<Vec<u8>>, EncodeError>> {
        let mut g = ffi::te_geometry { stripe_size: 0, num_stripes: 0, chunk_size: 0, sub_chunk_size: 0, slice_len: 0 };
        unsafe { ffi::te_slicer_geometry(self.raw.as_ptr(), data.len(), &mut g) };
        let sl = g.slice_len as usize;
        let mut out = vec![0u8; self.n() * sl];
        let c = cfg.ffi();
        let r = unsafe { ffi::te_slicer_encode(self.raw.as_ptr(), &c, data.as_ptr(), data.len(), out.as_mut_ptr(), out.len()) };
        Some(encode_status(r).map(|_| out.chunks(sl).map(<[u8]>::to_vec).collect()))
    }

    /// Slicer::decode (slicer.rs:298-364) in one te_slicer_decode; slices are (slice index, bytes).
    fn decode_object(&mut self, cfg: &ObjectCfg, slices: &[(usize, &[u8])]) -> Option<Result<Vec<u8>, DecodeError>> {
        if slices.len() < self.k { return Some(Err(DecodeError::NotEnoughSlices)) }
        let slen = slices[0].1.len();
        let mut ptrs = vec![std::ptr::null::<u8>(); self.n()];
        for (i, s) in slices {
            if *i >= self.n() || s.len() != slen { return Some(Err(DecodeError::InvalidLayout)) }
            ptrs[*i] = s.as_ptr();
        }
        // the blob is at most k chunks of every stripe: (slice_len - 48) * k bytes
        let mut out = vec![0u8; slen.saturating_sub(ffi::TE_META_SIZE as usize) * self.k + 1];
        let mut got = 0usize;
        let c = cfg.ffi();
        let r = unsafe {
            ffi::te_slicer_decode(self.raw.as_ptr(), &c, ptrs.as_ptr(), slen, out.as_mut_ptr(), out.len(), &mut got)
        };
        Some(decode_status(r).map(|_| {
            out.truncate(got);
            out
        }))
    }
}

/// RepairPlan (repair.rs:16-28) with the reference's public fields, read back from the library's
/// plan when it is built, so callers that walk `plan.stripes` (the node's per_helper_reqs,
/// network/node/src/features/spool/repair.rs:468-491) read it unchanged; the library handle it was
/// read from is kept for extract / repair.
pub struct RepairPlan {
    /// The slice being repaired.
    pub lost: SliceIndex,
    /// Number of stripes in the blob.
    pub num_stripes: u32,
    /// Full chunk size per stripe (bytes).
    pub chunk_size: u64,
    /// Sub-chunk size (chunk_size / alpha).
    pub sub_chunk_size: u64,
    /// Per-stripe repair plans.
    pub stripes: Vec<StripeRepair>,
    raw: *mut ffi::te_repair_plan,
}
/// StripeRepair (repair.rs:30-38).
pub struct StripeRepair { pub stripe: u32, pub lost_shard: SliceIndex, pub helpers: Vec<HelperPlan> }
/// HelperPlan (repair.rs:40-47).
pub struct HelperPlan { pub slice: SliceIndex, pub shard: SliceIndex, pub sub_chunks: Vec<u32> }
impl Drop for RepairPlan { fn drop(&mut self) { unsafe { ffi::te_repair_plan_free(self.raw) } } }
unsafe impl Send for RepairPlan {}

impl RepairPlan {
    /// The pub fields from the library's plan (te_repair_plan_get_info + te_repair_plan_stripe).
    fn wrap(raw: *mut ffi::te_repair_plan) -> Self {
        let mut info = ffi::te_repair_plan_info { lost: 0, num_stripes: 0, d: 0, beta: 0, chunk_size: 0, sub_chunk_size: 0 };
        unsafe { ffi::te_repair_plan_get_info(raw, &mut info) };
        let (d, beta) = (info.d as usize, info.beta as usize);
        let mut stripes = Vec::with_capacity(info.num_stripes as usize);
        for s in 0..info.num_stripes {
            let (mut lost_shard, mut slices, mut shards, mut subs) = (0u32, vec![0u32; d], vec![0u32; d], vec![0u32; d * beta]);
            unsafe {
                ffi::te_repair_plan_stripe(raw, s, &mut lost_shard, slices.as_mut_ptr(), shards.as_mut_ptr(), subs.as_mut_ptr())
            };
            let helpers = (0..d)
                .map(|h| HelperPlan { slice: SliceIndex::new(slices[h] as usize), shard: SliceIndex::new(shards[h] as usize),
                                      sub_chunks: subs[h * beta..(h + 1) * beta].to_vec() })
                .collect();
            stripes.push(StripeRepair { stripe: s, lost_shard: SliceIndex::new(lost_shard as usize), helpers });
        }
        Self { lost: SliceIndex::new(info.lost as usize), num_stripes: info.num_stripes, chunk_size: info.chunk_size,
               sub_chunk_size: info.sub_chunk_size, stripes, raw }
    }

    /// Slicer::repair_plan_from_params (repair.rs:137-201): blob_len / stripe_size from TrackInfo.
    pub fn from_params(coder: &ClayCoder, rotated: bool, lost: SliceIndex, available: &[SliceIndex], blob_len: u64,
                       stripe_size: u64) -> Result<Self, RepairError> {
        let av: Vec<u32> = available.iter().map(|s| **s as u32).collect();
        let mut p = std::ptr::null_mut();
        let r = unsafe {
            ffi::te_repair_plan_from_params(coder.raw.as_ptr(), rotated as i32, *lost as u32, av.as_ptr(), av.len(),
                                            blob_len, stripe_size, &mut p)
        };
        repair_status(r, None)?;
        Ok(Self::wrap(p))
    }
    /// Slicer::repair_plan (repair.rs:203-281): geometry from a reference slice's suffix.
    pub fn from_slice(coder: &ClayCoder, rotated: bool, lost: SliceIndex, available: &[SliceIndex], reference: &[u8])
            -> Result<Self, RepairError> {
        let av: Vec<u32> = available.iter().map(|s| **s as u32).collect();
        let mut p = std::ptr::null_mut();
        let r = unsafe {
            ffi::te_repair_plan_from_slice(coder.raw.as_ptr(), rotated as i32, *lost as u32, av.as_ptr(), av.len(),
                                           reference.as_ptr(), reference.len(), &mut p)
        };
        repair_status(r, None)?;
        Ok(Self::wrap(p))
    }

    /// extract_repair_data (repair.rs:97-130): the helper-side gather of its planned sub-chunks.
    pub fn extract(&self, slice: &[u8], helper: SliceIndex) -> Result<Vec<u8>, RepairError> {
        let n = unsafe { ffi::te_extract_repair_data_size(self.raw, *helper as u32) };
        let mut out = vec![0u8; n];
        let mut got = 0usize;
        let r = unsafe {
            ffi::te_extract_repair_data(self.raw, slice.as_ptr(), slice.len(), *helper as u32, out.as_mut_ptr(), out.len(),
                                        &mut got)
        };
        repair_status(r, None)?;
        out.truncate(got);
        Ok(out)
    }

    /// Slicer::repair (repair.rs:324-367): the lost slice (chunks + 48-byte suffix) from the
    /// helpers' extracts, indexed by slice id.
    pub fn repair(&self, coder: &mut ClayCoder, helpers: &[(SliceIndex, &[u8])], metadata: &[u8]) -> Result<Vec<u8>, RepairError> {
        let n = coder.n();
        let mut ptrs = vec![std::ptr::null::<u8>(); n];
        let mut lens = vec![0usize; n];
        for (i, d) in helpers {
            if **i >= n { return Err(RepairError::InvalidSlice) }
            ptrs[**i] = d.as_ptr();
            lens[**i] = d.len();
        }
        let mut out = vec![0u8; self.num_stripes as usize * self.chunk_size as usize + ffi::TE_META_SIZE as usize];
        let r = unsafe {
            ffi::te_slicer_repair(coder.raw.as_ptr(), self.raw, ptrs.as_ptr(), lens.as_ptr(), metadata.as_ptr(),
                                  out.as_mut_ptr(), out.len())
        };
        repair_status(r, None)?;
        Ok(out)
    }
}
