//! `quack` — drop-in replacement for the `quack/` submodule of ygina/sidekick,
//! backed by the MI355X engine `libquack_hip.so` (C ABI: `include/quack_hip.h`).
//!
//! The callers keep their code:
//! `use quack::{PowerSumQuack, PowerSumQuackU32}` (`sidekick.rs:9`,
//! `sidekick_multi.rs:11`), `use quack::arithmetic::{self, ModularArithmetic}`
//! and the strawmen (`media_client.rs:21-22`), `bincode::serialize(&quack)`
//! (`sidekick.rs:187`) / `bincode::deserialize::<PowerSumQuackU32>`
//! (`media_client.rs:227`).
//!
//! Per-packet calls (`insert`, `remove`, `sub_assign`, `to_coeffs`, `eval`)
//! run on the host inside libquack_hip (a kernel launch costs more than one
//! insert).  The batch calls (`insert_batch*`, `decode_*_device`, packet and
//! flow batches, the sharded calls of [`Comm`]) run the gfx950 kernels and
//! return [`QuackError`] with `QK_E_NO_DEVICE` when there is no GPU — there is
//! no CPU fallback.

pub mod arithmetic;
pub mod ffi;
#[cfg(feature = "strawmen")]
mod strawmen;
#[cfg(feature = "strawmen")]
pub use strawmen::{StrawmanAQuack, StrawmanBQuack};

use arithmetic::{Field, ModularInteger};
use serde::{Deserialize, Deserializer, Serialize, Serializer};
use std::ffi::CStr;
use std::fmt;
use std::marker::PhantomData;
use std::os::raw::{c_int, c_void};
use std::ptr;

pub type CoefficientVector<T> = Vec<ModularInteger<T>>;

/// A non-zero status of libquack_hip.
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub struct QuackError {
    pub status: i32,
}

impl fmt::Display for QuackError {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        let msg = unsafe { CStr::from_ptr(ffi::qk_strerror(self.status)) };
        write!(f, "quack: {} ({})", msg.to_string_lossy(), self.status)
    }
}

impl std::error::Error for QuackError {}

pub type Result<T> = std::result::Result<T, QuackError>;

fn check(rc: c_int) -> Result<()> {
    if rc == ffi::QK_OK { Ok(()) } else { Err(QuackError { status: rc }) }
}

/// The crate's infallible surface panics where the original crate panics
/// (threshold mismatch, undecodable difference, insert into `new(0)`).
fn ok(rc: c_int) {
    if let Err(e) = check(rc) {
        panic!("{}", e);
    }
}

/// Library version string (`quack-hip …`).
/// The distinct roots in GF(p32), ascending, of the polynomial `coeffs`
/// describes (`to_coeffs`): a log entry is a root-test hit (`media_client.rs:310`)
/// exactly when it is congruent to one of them (`qk_u32_roots`).
pub fn roots_u32(coeffs: &[u32]) -> Result<Vec<u32>> {
    let mut out = vec![0u32; coeffs.len().max(1)];
    let mut k = 0u32;
    check(unsafe { ffi::qk_u32_roots(coeffs.as_ptr(), coeffs.len() as u32, out.as_mut_ptr(), out.len() as u32, &mut k) })?;
    out.truncate(k as usize);
    Ok(out)
}

/// [`roots_u32`] over GF(p64) (`qk_u64_roots`).
pub fn roots_u64(coeffs: &[u64]) -> Result<Vec<u64>> {
    let mut out = vec![0u64; coeffs.len().max(1)];
    let mut k = 0u32;
    check(unsafe { ffi::qk_u64_roots(coeffs.as_ptr(), coeffs.len() as u32, out.as_mut_ptr(), out.len() as u32, &mut k) })?;
    out.truncate(k as usize);
    Ok(out)
}

pub fn version() -> String {
    unsafe { CStr::from_ptr(ffi::qk_version()) }.to_string_lossy().into_owned()
}

/// The sketch trait every caller imports (`use quack::PowerSumQuack`).
pub trait PowerSumQuack: Clone {
    type Element: Copy + PartialEq;
    /// An empty sketch that can decode up to `threshold` missing ids.
    fn new(threshold: usize) -> Self;
    fn threshold(&self) -> usize;
    /// Inserts minus removes, wrapping.
    fn count(&self) -> u32;
    /// The last inserted id (unchanged by `remove` and `sub_assign`).
    fn last_value(&self) -> Option<Self::Element>;
    fn insert(&mut self, value: Self::Element);
    fn remove(&mut self, value: Self::Element);
    /// `self -= rhs` (`media_client.rs:296`).
    fn sub_assign(&mut self, rhs: Self);
    /// Newton's identities: the coefficients c1..cd (d = count) of the
    /// polynomial whose roots are the missing ids (`media_client.rs:304`).
    fn to_coeffs(&self) -> CoefficientVector<Self::Element>;
    /// The entries of `log` that are missing (every entry congruent to a
    /// root, in log order).
    fn decode_with_log(&self, log: &[Self::Element]) -> Vec<Self::Element>;
}

/// Device context of one GPU: scratch memory, streams, profiling events.
pub struct Context {
    raw: *mut ffi::qk_ctx,
    owned: bool,
}

unsafe impl Send for Context {}

impl Context {
    pub fn new(device: i32) -> Result<Context> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::qk_ctx_create(device, &mut raw) })?;
        Ok(Context { raw, owned: true })
    }
    pub fn device_count() -> Result<i32> {
        let mut n: c_int = 0;
        check(unsafe { ffi::qk_device_count(&mut n) })?;
        Ok(n)
    }
    pub fn as_raw(&self) -> *mut ffi::qk_ctx {
        self.raw
    }
    /// Waits for the context's work (and `stream`'s, if not null).
    pub fn synchronize(&self, stream: *mut c_void) -> Result<()> {
        check(unsafe { ffi::qk_ctx_synchronize(self.raw, stream) })
    }
    /// HIP-event timing of every dominant-kernel launch while on.
    pub fn set_profiling(&self, on: bool) -> Result<()> {
        check(unsafe { ffi::qk_ctx_set_profiling(self.raw, on as c_int) })
    }
    /// (summed kernel milliseconds, launches) since the last call.
    pub fn kernel_stats(&self) -> Result<(f64, u64)> {
        let (mut ms, mut n) = (0f64, 0u64);
        check(unsafe { ffi::qk_ctx_kernel_stats(self.raw, &mut ms, &mut n) })?;
        Ok((ms, n))
    }
    pub fn set_grid(&self, blocks: u32) -> Result<()> {
        check(unsafe { ffi::qk_ctx_set_grid(self.raw, blocks) })
    }
    /// A measurement knob (`qk_ctx_set_knob`).
    pub fn set_knob(&self, name: &str, value: i64) -> Result<()> {
        let c = std::ffi::CString::new(name).map_err(|_| QuackError { status: ffi::QK_E_INVAL })?;
        check(unsafe { ffi::qk_ctx_set_knob(self.raw, c.as_ptr(), value) })
    }
    /// Frees retired scratch (a device-wide synchronisation).
    pub fn trim(&self) -> Result<()> {
        check(unsafe { ffi::qk_ctx_trim(self.raw) })
    }
}

impl Drop for Context {
    fn drop(&mut self) {
        if self.owned {
            unsafe { ffi::qk_ctx_destroy(self.raw) }
        }
    }
}

/// Page-locked host memory (`qk_host_alloc`): a sniffer that writes ids here
/// has them DMA'd to the GPU without a staging copy.
pub struct PinnedBuffer<T: Copy> {
    ptr: *mut T,
    len: usize,
}

unsafe impl<T: Copy + Send> Send for PinnedBuffer<T> {}

impl<T: Copy + Default> PinnedBuffer<T> {
    pub fn new(len: usize) -> Result<Self> {
        let mut p: *mut c_void = ptr::null_mut();
        check(unsafe { ffi::qk_host_alloc(len.max(1) * std::mem::size_of::<T>(), &mut p) })?;
        let ptr = p as *mut T;
        for i in 0..len {
            unsafe { ptr.add(i).write(T::default()) };
        }
        Ok(PinnedBuffer { ptr, len })
    }
}

impl<T: Copy> std::ops::Deref for PinnedBuffer<T> {
    type Target = [T];
    fn deref(&self) -> &[T] {
        unsafe { std::slice::from_raw_parts(self.ptr, self.len) }
    }
}

impl<T: Copy> std::ops::DerefMut for PinnedBuffer<T> {
    fn deref_mut(&mut self) -> &mut [T] {
        unsafe { std::slice::from_raw_parts_mut(self.ptr, self.len) }
    }
}

impl<T: Copy> Drop for PinnedBuffer<T> {
    fn drop(&mut self) {
        unsafe { ffi::qk_host_free(self.ptr as *mut c_void) };
    }
}

/// Calls `f(cap, &mut n)` with a growing hit buffer until it fits.
fn with_hits(first_cap: usize, mut f: impl FnMut(*mut u64, usize, &mut usize) -> c_int) -> Result<Vec<u64>> {
    let mut cap = first_cap.max(1);
    loop {
        let mut hits = vec![0u64; cap];
        let mut n = 0usize;
        let rc = f(hits.as_mut_ptr(), cap, &mut n);
        if rc == ffi::QK_E_CAPACITY && n > cap {
            cap = n;
            continue;
        }
        check(rc)?;
        hits.truncate(n);
        return Ok(hits);
    }
}

/// Generates PowerSumQuackU32 / PowerSumQuackU64 over their C state.
macro_rules! power_sum_quack {
    ($name:ident, $wire:ident, $elem:ty, $raw:ty, $word:ty, hdr = $hdr:expr,
     size = $size:path, init = $init:path, insert = $insert:path, remove = $remove:path,
     sub_assign = $sub:path, merge = $merge:path, to_coeffs = $coeffs:path,
     decode_host = $dhost:path, encode_host = $ehost:path, encode_device = $edev:path,
     decode_device = $ddev:path, root_test_device = $rtdev:path,
     encode_sharded = $esh:path, decode_sharded = $dsh:path) => {
        /// Power-sum quACK: `threshold` power sums of the inserted ids over
        /// GF(p), the count and the last inserted id.  The bytes are the C
        /// state (header words, then the sums), so `Clone` is a copy.
        #[derive(Clone, PartialEq, Eq)]
        pub struct $name {
            words: Vec<$word>,
        }

        impl $name {
            fn raw(&self) -> *const $raw {
                self.words.as_ptr() as *const $raw
            }
            fn raw_mut(&mut self) -> *mut $raw {
                self.words.as_mut_ptr() as *mut $raw
            }
            fn state(&self) -> &$raw {
                unsafe { &*self.raw() }
            }
            fn with_threshold(threshold: u32) -> Result<Self> {
                let bytes = unsafe { $size(threshold) };
                let mut q = $name { words: vec![0; bytes / std::mem::size_of::<$word>()] };
                check(unsafe { $init(q.raw_mut(), threshold) })?;
                Ok(q)
            }
            /// The canonical power sums S_1..S_t (after the header words).
            pub fn power_sums(&self) -> &[$elem] {
                &self.words[$hdr..]
            }
            /// Append a stream that followed this one (additivity): sums and
            /// counts add, `last_value` from `later` if it has one.
            pub fn merge(&mut self, later: &Self) -> Result<()> {
                check(unsafe { $merge(self.raw_mut(), later.raw()) })
            }

            /// Insert every id of a host slice in order, on the GPU (chunked
            /// pinned H2D overlapped with the encode kernel).
            pub fn insert_batch(&mut self, ctx: &Context, ids: &[$elem]) -> Result<()> {
                check(unsafe { $ehost(ctx.raw, ids.as_ptr(), ids.len(), self.raw_mut()) })
            }
            /// Insert `n` device-resident ids in order (the HBM-resident path).
            ///
            /// # Safety
            /// `d_ids` must point to `n` ids in device memory of `ctx`'s GPU;
            /// `stream` is a `hipStream_t` of that device or null.
            pub unsafe fn insert_batch_device(&mut self, ctx: &Context, d_ids: *const $elem, n: usize,
                                              stream: *mut c_void) -> Result<()> {
                check($edev(ctx.raw, d_ids, n, self.raw_mut(), stream))
            }

            /// Positions of the missing entries of a host log (CPU root test),
            /// cut at the first entry equal to `last_value()` when
            /// `stop_at_last` (`media_client.rs:304-313`).
            pub fn decode_positions(&self, log: &[$elem], stop_at_last: bool) -> Result<Vec<u64>> {
                with_hits(self.threshold(), |h, cap, n| unsafe {
                    $dhost(self.raw(), log.as_ptr(), log.len(), stop_at_last as c_int, h, cap, n)
                })
            }
            /// The same over a device-resident log (gfx950 root test).
            ///
            /// # Safety
            /// `d_log` must point to `n` ids in device memory of `ctx`'s GPU.
            pub unsafe fn decode_positions_device(&self, ctx: &Context, d_log: *const $elem, n: usize,
                                                  stop_at_last: bool, stream: *mut c_void) -> Result<Vec<u64>> {
                with_hits(self.threshold().max(64), |h, cap, nh| {
                    $ddev(ctx.raw, self.raw(), d_log, n, stop_at_last as c_int, h, cap, nh, stream)
                })
            }
            /// Root test of explicit coefficients over a device-resident log;
            /// `stop_value` reproduces the `break` at `media_client.rs:307-309`.
            ///
            /// # Safety
            /// As [`Self::decode_positions_device`].
            pub unsafe fn root_test_device(ctx: &Context, coeffs: &[ModularInteger<$elem>], d_log: *const $elem,
                                           n: usize, stop_value: Option<$elem>, stream: *mut c_void)
                                           -> Result<Vec<u64>> {
                use arithmetic::ModularArithmetic;
                let c: Vec<$elem> = coeffs.iter().map(|m| m.value()).collect();
                with_hits(c.len().max(64), |h, cap, nh| {
                    $rtdev(ctx.raw, c.as_ptr(), c.len() as u32, d_log, n, stop_value.is_some() as c_int,
                           stop_value.unwrap_or(0), h, cap, nh, stream)
                })
            }

            /// Sharded encode over the communicator's GPUs: local rank i
            /// encodes `d_ids[i][..n[i]]`, one RCCL reduce merges the shards on
            /// global rank `root`, which appends the stream to `self`.
            ///
            /// # Safety
            /// Each `d_ids[i]` must be device memory of local rank i's GPU.
            pub unsafe fn insert_batch_sharded(&mut self, comm: &Comm, d_ids: &[*const $elem], n: &[usize],
                                               root: i32) -> Result<()> {
                comm.check_local(d_ids.len(), n.len())?;
                check($esh(comm.raw, d_ids.as_ptr(), n.as_ptr(), self.raw_mut(), root, ptr::null()))
            }
            /// Sharded decode: every rank gets the global positions of the
            /// missing entries of the log cut into shards (one per local rank).
            ///
            /// # Safety
            /// Each `d_log[i]` must be device memory of local rank i's GPU.
            pub unsafe fn decode_positions_sharded(&self, comm: &Comm, root: i32, d_log: &[*const $elem],
                                                   n: &[usize], stop_at_last: bool) -> Result<Vec<u64>> {
                comm.check_local(d_log.len(), n.len())?;
                with_hits(self.threshold().max(64), |h, cap, nh| {
                    $dsh(comm.raw, self.raw(), root, d_log.as_ptr(), n.as_ptr(), stop_at_last as c_int, h, cap,
                         nh, ptr::null())
                })
            }

            fn to_wire(&self) -> $wire {
                $wire {
                    power_sums: self.power_sums().iter().map(|&v| ModularInteger::from_canonical(v)).collect(),
                    last_value: self.last_value(),
                    count: self.count(),
                }
            }
            fn from_wire(w: $wire) -> std::result::Result<Self, String> {
                use arithmetic::ModularArithmetic;
                let mut q = Self::with_threshold(w.power_sums.len() as u32).map_err(|e| e.to_string())?;
                for (i, m) in w.power_sums.iter().enumerate() {
                    if m.value() >= <$elem as Field>::MODULUS {
                        return Err(format!("power sum {} is not canonical", i));
                    }
                    q.words[$hdr + i] = m.value();
                }
                let st = unsafe { &mut *q.raw_mut() };
                st.count = w.count;
                st.has_last = w.last_value.is_some() as u32;
                st.last_value = w.last_value.unwrap_or(0);
                Ok(q)
            }
        }

        impl PowerSumQuack for $name {
            type Element = $elem;
            fn new(threshold: usize) -> Self {
                assert!(threshold <= u32::MAX as usize, "threshold too large");
                Self::with_threshold(threshold as u32).unwrap_or_else(|e| panic!("{}", e))
            }
            fn threshold(&self) -> usize {
                self.state().threshold as usize
            }
            fn count(&self) -> u32 {
                self.state().count
            }
            fn last_value(&self) -> Option<$elem> {
                let s = self.state();
                if s.has_last != 0 { Some(s.last_value) } else { None }
            }
            fn insert(&mut self, value: $elem) {
                ok(unsafe { $insert(self.raw_mut(), value) })
            }
            fn remove(&mut self, value: $elem) {
                ok(unsafe { $remove(self.raw_mut(), value) })
            }
            fn sub_assign(&mut self, rhs: Self) {
                ok(unsafe { $sub(self.raw_mut(), rhs.raw()) })
            }
            fn to_coeffs(&self) -> CoefficientVector<$elem> {
                let mut c: Vec<$elem> = vec![0; self.threshold().max(1)];
                let mut d = 0u32;
                ok(unsafe { $coeffs(self.raw(), c.as_mut_ptr(), c.len() as u32, &mut d) });
                c.truncate(d as usize);
                c.into_iter().map(ModularInteger::from_canonical).collect()
            }
            fn decode_with_log(&self, log: &[$elem]) -> Vec<$elem> {
                if self.count() == 0 {
                    return vec![];
                }
                let pos = self.decode_positions(log, false).unwrap_or_else(|e| panic!("{}", e));
                pos.into_iter().map(|i| log[i as usize]).collect()
            }
        }

        impl fmt::Debug for $name {
            fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
                f.debug_struct(stringify!($name))
                    .field("power_sums", &self.power_sums())
                    .field("last_value", &self.last_value())
                    .field("count", &self.count())
                    .finish()
            }
        }

        /// The serde shape of the original crate's derived struct: bincode
        /// writes the sums as a u64 length + values, the Option tag + value,
        /// then the count (the bytes `qk_*_serialize` produces).
        #[derive(Serialize, Deserialize)]
        struct $wire {
            power_sums: Vec<ModularInteger<$elem>>,
            last_value: Option<$elem>,
            count: u32,
        }

        impl Serialize for $name {
            fn serialize<S: Serializer>(&self, s: S) -> std::result::Result<S::Ok, S::Error> {
                self.to_wire().serialize(s)
            }
        }

        impl<'de> Deserialize<'de> for $name {
            fn deserialize<D: Deserializer<'de>>(d: D) -> std::result::Result<Self, D::Error> {
                let w = $wire::deserialize(d)?;
                $name::from_wire(w).map_err(serde::de::Error::custom)
            }
        }
    };
}

power_sum_quack!(PowerSumQuackU32, WireU32, u32, ffi::qk_u32, u32, hdr = 4,
    size = ffi::qk_u32_size, init = ffi::qk_u32_init, insert = ffi::qk_u32_insert, remove = ffi::qk_u32_remove,
    sub_assign = ffi::qk_u32_sub_assign, merge = ffi::qk_u32_merge, to_coeffs = ffi::qk_u32_to_coeffs,
    decode_host = ffi::qk_u32_decode_host, encode_host = ffi::qk_u32_encode_host,
    encode_device = ffi::qk_u32_encode_device, decode_device = ffi::qk_u32_decode_device,
    root_test_device = ffi::qk_u32_root_test_device,
    encode_sharded = ffi::qk_u32_encode_sharded, decode_sharded = ffi::qk_u32_decode_sharded);

power_sum_quack!(PowerSumQuackU64, WireU64, u64, ffi::qk_u64, u64, hdr = 3,
    size = ffi::qk_u64_size, init = ffi::qk_u64_init, insert = ffi::qk_u64_insert, remove = ffi::qk_u64_remove,
    sub_assign = ffi::qk_u64_sub_assign, merge = ffi::qk_u64_merge, to_coeffs = ffi::qk_u64_to_coeffs,
    decode_host = ffi::qk_u64_decode_host, encode_host = ffi::qk_u64_encode_host,
    encode_device = ffi::qk_u64_encode_device, decode_device = ffi::qk_u64_decode_device,
    root_test_device = ffi::qk_u64_root_test_device,
    encode_sharded = ffi::qk_u64_encode_sharded, decode_sharded = ffi::qk_u64_decode_sharded);

impl PowerSumQuackU32 {
    /// One sniffer ring fill of `n` captured `stride`-byte records (plus
    /// optional `sockaddr_ll` metadata) in device memory, filtered and
    /// inserted exactly as the per-packet loop of `sidekick.rs:76-124` would;
    /// a reset datagram to `my_ipv4` restarts the sketch.
    ///
    /// # Safety
    /// `d_bufs` (n * stride bytes) and `d_meta` (n records or null) must be
    /// device memory of `ctx`'s GPU.
    pub unsafe fn insert_packets_device(&mut self, ctx: &Context, d_bufs: *const u8, n: usize, stride: usize,
                                        d_meta: *const ffi::qk_pkt_meta, my_ipv4: Option<[u8; 4]>,
                                        stream: *mut c_void) -> Result<ffi::qk_pkt_stats> {
        let mut st = ffi::qk_pkt_stats::default();
        let ip = my_ipv4.as_ref().map_or(ptr::null(), |a| a.as_ptr());
        check(ffi::qk_u32_encode_packets_device(ctx.raw, d_bufs, n, stride, d_meta, ip, self.raw_mut(), &mut st,
                                                stream))?;
        Ok(st)
    }
}

/// One sketch per flow for a packet batch (`SidekickMulti`,
/// `sidekick_multi.rs:65-90,101-143`): the batch's flows in ascending key
/// order.  When `stats.resets > 0` the caller clears its table before merging
/// (the sniff loops' `senders = HashMap::new()`, `sidekick_multi.rs:205,265`).
pub struct FlowBatch {
    pub flows: Vec<(ffi::qk_flow_key, PowerSumQuackU32)>,
    pub stats: ffi::qk_pkt_stats,
}

/// # Safety
/// `d_bufs` (n * stride bytes) and `d_meta` (n records or null) must be device
/// memory of `ctx`'s GPU.
pub unsafe fn encode_flows_device(ctx: &Context, d_bufs: *const u8, n: usize, stride: usize,
                                  d_meta: *const ffi::qk_pkt_meta, my_addr: Option<[u8; 6]>, threshold: u32,
                                  stream: *mut c_void) -> Result<FlowBatch> {
    let rsz = ffi::qk_u32_size(threshold);
    let words = rsz / 4;
    let addr = my_addr.as_ref().map_or(ptr::null(), |a| a.as_ptr());
    let mut cap = 1024usize;
    loop {
        let mut keys = vec![ffi::qk_flow_key::default(); cap];
        let mut sketches = vec![0u32; cap * words];
        let (mut nf, mut st) = (0usize, ffi::qk_pkt_stats::default());
        let rc = ffi::qk_u32_encode_flows_device(ctx.raw, d_bufs, n, stride, d_meta, addr, threshold,
                                                 keys.as_mut_ptr(), sketches.as_mut_ptr() as *mut u8, cap,
                                                 &mut nf, &mut st, stream);
        if rc == ffi::QK_E_CAPACITY && nf > cap {
            cap = nf;
            continue;
        }
        check(rc)?;
        let flows = (0..nf)
            .map(|i| (keys[i], PowerSumQuackU32 { words: sketches[i * words..(i + 1) * words].to_vec() }))
            .collect();
        return Ok(FlowBatch { flows, stats: st });
    }
}

/// Multi-GPU communicator over RCCL (xGMI): one process driving several
/// GPUs ([`Comm::new`]) or one process per GPU ([`Comm::init_rank`]).
pub struct Comm {
    raw: *mut ffi::qk_comm,
    nlocal: usize,
}

unsafe impl Send for Comm {}

impl Comm {
    /// One process, local rank i on `devices[i]` (ncclCommInitAll).
    pub fn new(devices: &[i32]) -> Result<Comm> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::qk_comm_create(devices.len() as c_int, devices.as_ptr(), &mut raw) })?;
        Ok(Comm { raw, nlocal: devices.len() })
    }
    /// The id rank 0 creates and ships to the other processes.
    pub fn unique_id() -> Result<[u8; ffi::QK_COMM_ID_BYTES]> {
        let mut id = [0u8; ffi::QK_COMM_ID_BYTES];
        check(unsafe { ffi::qk_comm_unique_id(id.as_mut_ptr()) })?;
        Ok(id)
    }
    /// One process per GPU.
    pub fn init_rank(id: &[u8; ffi::QK_COMM_ID_BYTES], rank: i32, world: i32, device: i32) -> Result<Comm> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::qk_comm_init_rank(id.as_ptr(), rank, world, device, &mut raw) })?;
        Ok(Comm { raw, nlocal: 1 })
    }
    /// (world, local ranks, global rank of local rank 0)
    pub fn info(&self) -> Result<(i32, i32, i32)> {
        let (mut w, mut l, mut f) = (0, 0, 0);
        check(unsafe { ffi::qk_comm_info(self.raw, &mut w, &mut l, &mut f) })?;
        Ok((w, l, f))
    }
    /// One rank whose collectives run through a host channel (`ops`) instead
    /// of RCCL: the same protocol, e.g. more ranks than GPUs.
    ///
    /// # Safety
    /// The callbacks must implement the collectives over all ranks and stay
    /// valid (with `ops.user`) until the communicator is dropped.
    pub unsafe fn init_host(ops: &ffi::qk_comm_host_ops, rank: i32, world: i32, device: i32) -> Result<Comm> {
        let mut raw = ptr::null_mut();
        check(ffi::qk_comm_init_host(ops, rank, world, device, &mut raw))?;
        Ok(Comm { raw, nlocal: 1 })
    }
    /// The context of a local rank, owned by the communicator: the borrow
    /// keeps the communicator (and so the context) alive.
    pub fn context(&self, local: i32) -> Result<ContextRef<'_>> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::qk_comm_context(self.raw, local, &mut raw) })?;
        Ok(ContextRef { ctx: Context { raw, owned: false }, _comm: PhantomData })
    }
    pub fn barrier(&self) -> Result<()> {
        check(unsafe { ffi::qk_comm_barrier(self.raw) })
    }
    /// Bound (ms, 0 = none) on every wait for an RCCL collective; past it the
    /// communicator aborts and the call returns QK_E_COMM.
    pub fn set_timeout(&self, ms: i64) -> Result<()> {
        check(unsafe { ffi::qk_comm_set_timeout(self.raw, ms) })
    }
    /// (ranks, device, rank) as RCCL reports them for local rank `local`.
    pub fn rccl_info(&self, local: i32) -> Result<(i32, i32, i32)> {
        let (mut k, mut d, mut r) = (0, 0, 0);
        check(unsafe { ffi::qk_comm_rccl_info(self.raw, local, &mut k, &mut d, &mut r) })?;
        Ok((k, d, r))
    }
    fn check_local(&self, a: usize, b: usize) -> Result<()> {
        if a != self.nlocal || b != self.nlocal {
            return Err(QuackError { status: ffi::QK_E_INVAL });
        }
        Ok(())
    }
}

/// A communicator-owned [`Context`], borrowed from its [`Comm`].
pub struct ContextRef<'a> {
    ctx: Context,
    _comm: PhantomData<&'a Comm>,
}

impl std::ops::Deref for ContextRef<'_> {
    type Target = Context;
    fn deref(&self) -> &Context {
        &self.ctx
    }
}

impl Drop for Comm {
    fn drop(&mut self) {
        unsafe { ffi::qk_comm_destroy(self.raw) }
    }
}

#[cfg(test)]
mod tests {
    use super::arithmetic::{self, ModularArithmetic};
    use super::*;

    #[test]
    fn kat_small_stream() {
        // ids {1..5}, t = 4: S = [15, 55, 225, 979]
        let mut q = PowerSumQuackU32::new(4);
        for id in 1..=5u32 {
            q.insert(id);
        }
        assert_eq!(q.power_sums(), &[15, 55, 225, 979]);
        assert_eq!(q.count(), 5);
        assert_eq!(q.last_value(), Some(5));
    }

    #[test]
    fn decode_round_like_media_client() {
        // media_client.rs:247-319: sender sketch minus receiver sketch, then
        // the root test over the sent log.
        let log: Vec<u32> = (0..200u32).map(|i| i.wrapping_mul(2_654_435_761)).collect();
        let missing = [3usize, 77, 150];
        let mut sent = PowerSumQuackU32::new(8);
        let mut recv = PowerSumQuackU32::new(8);
        for (i, &id) in log.iter().enumerate() {
            sent.insert(id);
            if !missing.contains(&i) {
                recv.insert(id);
            }
        }
        let mut diff = sent.clone();
        diff.sub_assign(recv);
        assert_eq!(diff.count(), 3);
        let coeffs = diff.to_coeffs();
        let found: Vec<u32> = log.iter().copied().filter(|&x| arithmetic::eval(&coeffs, x).value() == 0).collect();
        assert_eq!(found, vec![log[3], log[77], log[150]]);
        assert_eq!(diff.decode_with_log(&log), found);
    }

    #[test]
    fn bincode_matches_c_image() {
        let mut q = PowerSumQuackU32::new(3);
        q.insert(7);
        q.insert(u32::MAX);
        let ours = bincode::serialize(&q).unwrap();
        let mut buf = vec![0u8; unsafe { ffi::qk_u32_serialized_size(q.raw()) }];
        let mut len = 0usize;
        assert_eq!(unsafe { ffi::qk_u32_serialize(q.raw(), buf.as_mut_ptr(), buf.len(), &mut len) }, 0);
        assert_eq!(&ours[..], &buf[..len]);
        let back: PowerSumQuackU32 = bincode::deserialize(&ours).unwrap();
        assert_eq!(back, q);
    }

    #[test]
    fn u64_field_and_modular_integer() {
        let mut q = PowerSumQuackU64::new(2);
        q.insert(u64::MAX);
        let x = ModularInteger::<u64>::new(u64::MAX);
        assert_eq!(q.power_sums(), &[x.value(), (x * x).value()]);
        assert_eq!((x * x.inv()).value(), 1);
    }
}
