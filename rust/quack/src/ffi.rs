//! Raw `extern "C"` declarations of `include/quack_hip.h` (libquack_hip.so).
//!
//! One declaration per prototype in the header, same order, same types
//! (`tests/test_rust_crate.py` parses both files and checks that every
//! header prototype appears here with the same parameter count and the
//! mapped types: `uint32_t` -> `u32`, `size_t` -> `usize`, `int` -> `c_int`,
//! `T *` -> `*mut T`, `const T *` -> `*const T`, `void *` -> `*mut c_void`,
//! `T *const *` -> `*const *mut T`, array parameters -> pointers).
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

pub const QK_P32: u32 = 4_294_967_291;
pub const QK_P64: u64 = 18_446_744_073_709_551_557;
pub const QK_MAX_THRESHOLD: u32 = 1024;
pub const QK_ID_OFFSET: usize = 63;
pub const QK_BUFFER_SIZE: usize = 67;
pub const QK_COMM_ID_BYTES: usize = 128;

pub const QK_OK: c_int = 0;
pub const QK_E_INVAL: c_int = -1;
pub const QK_E_THRESHOLD: c_int = -2;
pub const QK_E_MISMATCH: c_int = -3;
pub const QK_E_UNDECODABLE: c_int = -4;
pub const QK_E_CAPACITY: c_int = -5;
pub const QK_E_HIP: c_int = -6;
pub const QK_E_NO_DEVICE: c_int = -7;
pub const QK_E_NOMEM: c_int = -8;
pub const QK_E_FORMAT: c_int = -9;
pub const QK_E_COMM: c_int = -10;
pub const QK_E_PEER: c_int = -11;

/// `qk_u32`: header words then `threshold` canonical power sums.
#[repr(C)]
pub struct qk_u32 {
    pub threshold: u32,
    pub count: u32,
    pub has_last: u32,
    pub last_value: u32,
    pub power_sums: [u32; 0],
}

/// `qk_u64`: 16-byte header, `last_value`, then `threshold` power sums.
#[repr(C)]
pub struct qk_u64 {
    pub threshold: u32,
    pub count: u32,
    pub has_last: u32,
    pub reserved: u32,
    pub last_value: u64,
    pub power_sums: [u64; 0],
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct qk_pkt_meta {
    pub pkttype: u8,
    pub reserved: u8,
    pub protocol_be: u16,
    pub len: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub struct qk_pkt_stats {
    pub inserted: u64,
    pub discarded: u64,
    pub resets: u64,
    pub filtered: u64,
    pub last_reset_index: i64,
}

impl Default for qk_pkt_stats {
    fn default() -> Self {
        qk_pkt_stats { inserted: 0, discarded: 0, resets: 0, filtered: 0, last_reset_index: -1 }
    }
}

/// AddrKey (`sidekick_multi.rs:13`): src ip, src port, dst ip, dst port, wire order.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq, Hash, PartialOrd, Ord)]
pub struct qk_flow_key {
    pub addr: [u8; 12],
}

/// Opaque device context.
#[repr(C)]
pub struct qk_ctx {
    _private: [u8; 0],
}

/// Opaque multi-GPU communicator.
#[repr(C)]
pub struct qk_comm {
    _private: [u8; 0],
}

/// Host-channel collectives of `qk_comm_init_host` (each returns 0 on success).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct qk_comm_host_ops {
    pub user: *mut c_void,
    pub reduce_sum_u64: Option<unsafe extern "C" fn(user: *mut c_void, buf: *mut u64, n: usize, root: c_int) -> c_int>,
    pub broadcast_u64: Option<unsafe extern "C" fn(user: *mut c_void, buf: *mut u64, n: usize, root: c_int) -> c_int>,
    pub allgather_u64:
        Option<unsafe extern "C" fn(user: *mut c_void, send: *const u64, recv: *mut u64, n: usize) -> c_int>,
}

#[link(name = "quack_hip")]
extern "C" {
    pub fn qk_strerror(status: c_int) -> *const c_char;
    pub fn qk_version() -> *const c_char;

    // sketch state
    pub fn qk_u32_size(threshold: u32) -> usize;
    pub fn qk_u64_size(threshold: u32) -> usize;
    pub fn qk_u32_init(q: *mut qk_u32, threshold: u32) -> c_int;
    pub fn qk_u64_init(q: *mut qk_u64, threshold: u32) -> c_int;

    // host scalar path
    pub fn qk_u32_insert(q: *mut qk_u32, id: u32) -> c_int;
    pub fn qk_u64_insert(q: *mut qk_u64, id: u64) -> c_int;
    pub fn qk_u32_remove(q: *mut qk_u32, id: u32) -> c_int;
    pub fn qk_u64_remove(q: *mut qk_u64, id: u64) -> c_int;
    pub fn qk_u32_sub_assign(q: *mut qk_u32, rhs: *const qk_u32) -> c_int;
    pub fn qk_u64_sub_assign(q: *mut qk_u64, rhs: *const qk_u64) -> c_int;
    pub fn qk_u32_merge(q: *mut qk_u32, later: *const qk_u32) -> c_int;
    pub fn qk_u64_merge(q: *mut qk_u64, later: *const qk_u64) -> c_int;
    pub fn qk_u32_to_coeffs(q: *const qk_u32, coeffs: *mut u32, cap: u32, d: *mut u32) -> c_int;
    pub fn qk_u64_to_coeffs(q: *const qk_u64, coeffs: *mut u64, cap: u32, d: *mut u32) -> c_int;
    pub fn qk_u32_eval(coeffs: *const u32, d: u32, x: u32) -> u32;
    pub fn qk_u64_eval(coeffs: *const u64, d: u32, x: u64) -> u64;
    pub fn qk_u32_decode_host(diff: *const qk_u32, log: *const u32, n: usize, stop_at_last: c_int, hits: *mut u64,
                              cap: usize, n_hits: *mut usize) -> c_int;
    pub fn qk_u64_decode_host(diff: *const qk_u64, log: *const u64, n: usize, stop_at_last: c_int, hits: *mut u64,
                              cap: usize, n_hits: *mut usize) -> c_int;

    // bincode image
    pub fn qk_u32_serialized_size(q: *const qk_u32) -> usize;
    pub fn qk_u32_serialize(q: *const qk_u32, buf: *mut u8, cap: usize, len: *mut usize) -> c_int;
    pub fn qk_u32_deserialize(buf: *const u8, len: usize, q: *mut qk_u32, threshold_out: *mut u32) -> c_int;
    pub fn qk_u64_serialized_size(q: *const qk_u64) -> usize;
    pub fn qk_u64_serialize(q: *const qk_u64, buf: *mut u8, cap: usize, len: *mut usize) -> c_int;
    pub fn qk_u64_deserialize(buf: *const u8, len: usize, q: *mut qk_u64, threshold_out: *mut u32) -> c_int;

    // device context
    pub fn qk_device_count(n: *mut c_int) -> c_int;
    pub fn qk_ctx_create(device: c_int, out: *mut *mut qk_ctx) -> c_int;
    pub fn qk_ctx_destroy(ctx: *mut qk_ctx);
    pub fn qk_ctx_synchronize(ctx: *mut qk_ctx, stream: *mut c_void) -> c_int;
    pub fn qk_ctx_set_profiling(ctx: *mut qk_ctx, on: c_int) -> c_int;
    pub fn qk_ctx_kernel_stats(ctx: *mut qk_ctx, total_ms: *mut f64, launches: *mut u64) -> c_int;
    pub fn qk_ctx_trim(ctx: *mut qk_ctx) -> c_int;
    pub fn qk_ctx_set_grid(ctx: *mut qk_ctx, blocks: u32) -> c_int;
    pub fn qk_ctx_set_knob(ctx: *mut qk_ctx, name: *const c_char, value: i64) -> c_int;
    pub fn qk_clock_probe(ctx: *mut qk_ctx, microseconds: u32, d_out: *mut u64, stream: *mut c_void) -> c_int;
    pub fn qk_host_alloc(bytes: usize, out: *mut *mut c_void) -> c_int;
    pub fn qk_host_free(p: *mut c_void) -> c_int;

    // batch encode
    pub fn qk_u32_partial_words(threshold: u32) -> usize;
    pub fn qk_u64_partial_words(threshold: u32) -> usize;
    pub fn qk_u32_encode_device_async(ctx: *mut qk_ctx, d_ids: *const u32, n: usize, threshold: u32,
                                      d_partial: *mut u64, stream: *mut c_void) -> c_int;
    pub fn qk_u64_encode_device_async(ctx: *mut qk_ctx, d_ids: *const u64, n: usize, threshold: u32,
                                      d_partial: *mut u64, stream: *mut c_void) -> c_int;
    pub fn qk_u32_merge_partial(q: *mut qk_u32, partial: *const u64, has_last: c_int, last: u32) -> c_int;
    pub fn qk_u64_merge_partial(q: *mut qk_u64, partial: *const u64, has_last: c_int, last: u64) -> c_int;
    pub fn qk_u32_encode_device(ctx: *mut qk_ctx, d_ids: *const u32, n: usize, q: *mut qk_u32,
                                stream: *mut c_void) -> c_int;
    pub fn qk_u64_encode_device(ctx: *mut qk_ctx, d_ids: *const u64, n: usize, q: *mut qk_u64,
                                stream: *mut c_void) -> c_int;
    pub fn qk_u32_encode_host(ctx: *mut qk_ctx, h_ids: *const u32, n: usize, q: *mut qk_u32) -> c_int;
    pub fn qk_u64_encode_host(ctx: *mut qk_ctx, h_ids: *const u64, n: usize, q: *mut qk_u64) -> c_int;

    // packet batches and per-flow sketches
    pub fn qk_u32_encode_packets_device(ctx: *mut qk_ctx, d_bufs: *const u8, n: usize, stride: usize,
                                        d_meta: *const qk_pkt_meta, my_ipv4: *const u8, q: *mut qk_u32,
                                        stats: *mut qk_pkt_stats, stream: *mut c_void) -> c_int;
    pub fn qk_u32_encode_flows_device(ctx: *mut qk_ctx, d_bufs: *const u8, n: usize, stride: usize,
                                      d_meta: *const qk_pkt_meta, my_addr: *const u8, threshold: u32,
                                      keys: *mut qk_flow_key, sketches: *mut u8, cap: usize, n_flows: *mut usize,
                                      stats: *mut qk_pkt_stats, stream: *mut c_void) -> c_int;
    pub fn qk_u32_encode_segments_device(ctx: *mut qk_ctx, d_ids: *const u32, offsets: *const u64, nseg: usize,
                                         threshold: u32, sketches: *mut u8, stream: *mut c_void) -> c_int;

    // root test / decode
    pub fn qk_u32_root_test_device(ctx: *mut qk_ctx, coeffs: *const u32, d: u32, d_log: *const u32, n: usize,
                                   stop_at_value: c_int, stop_value: u32, hits: *mut u64, cap: usize,
                                   n_hits: *mut usize, stream: *mut c_void) -> c_int;
    pub fn qk_u64_root_test_device(ctx: *mut qk_ctx, coeffs: *const u64, d: u32, d_log: *const u64, n: usize,
                                   stop_at_value: c_int, stop_value: u64, hits: *mut u64, cap: usize,
                                   n_hits: *mut usize, stream: *mut c_void) -> c_int;
    pub fn qk_u32_root_test_shard_device(ctx: *mut qk_ctx, coeffs: *const u32, d: u32, d_log: *const u32, n: usize,
                                         stop_at_value: c_int, stop_value: u32, hits: *mut u64, cap: usize,
                                         n_hits: *mut usize, stop_index: *mut u64, stream: *mut c_void) -> c_int;
    pub fn qk_u64_root_test_shard_device(ctx: *mut qk_ctx, coeffs: *const u64, d: u32, d_log: *const u64, n: usize,
                                         stop_at_value: c_int, stop_value: u64, hits: *mut u64, cap: usize,
                                         n_hits: *mut usize, stop_index: *mut u64, stream: *mut c_void) -> c_int;
    pub fn qk_u32_roots(coeffs: *const u32, d: u32, roots: *mut u32, cap: u32, k: *mut u32) -> c_int;
    pub fn qk_u64_roots(coeffs: *const u64, d: u32, roots: *mut u64, cap: u32, k: *mut u32) -> c_int;
    pub fn qk_u32_decode_device(ctx: *mut qk_ctx, diff: *const qk_u32, d_log: *const u32, n: usize,
                                stop_at_last: c_int, hits: *mut u64, cap: usize, n_hits: *mut usize,
                                stream: *mut c_void) -> c_int;
    pub fn qk_u64_decode_device(ctx: *mut qk_ctx, diff: *const qk_u64, d_log: *const u64, n: usize,
                                stop_at_last: c_int, hits: *mut u64, cap: usize, n_hits: *mut usize,
                                stream: *mut c_void) -> c_int;

    // multi-GPU over RCCL
    pub fn qk_comm_unique_id(id: *mut u8) -> c_int;
    pub fn qk_comm_create(ndev: c_int, devices: *const c_int, out: *mut *mut qk_comm) -> c_int;
    pub fn qk_comm_init_rank(id: *const u8, rank: c_int, world: c_int, device: c_int,
                             out: *mut *mut qk_comm) -> c_int;
    pub fn qk_comm_init_host(ops: *const qk_comm_host_ops, rank: c_int, world: c_int, device: c_int,
                             out: *mut *mut qk_comm) -> c_int;
    pub fn qk_comm_destroy(comm: *mut qk_comm);
    pub fn qk_comm_info(comm: *const qk_comm, world: *mut c_int, nlocal: *mut c_int, first_rank: *mut c_int) -> c_int;
    pub fn qk_comm_context(comm: *mut qk_comm, local: c_int, out: *mut *mut qk_ctx) -> c_int;
    pub fn qk_comm_barrier(comm: *mut qk_comm) -> c_int;
    pub fn qk_comm_set_timeout(comm: *mut qk_comm, ms: i64) -> c_int;
    pub fn qk_comm_rccl_info(comm: *const qk_comm, local: c_int, count: *mut c_int, device: *mut c_int,
                             rank: *mut c_int) -> c_int;
    pub fn qk_u32_encode_sharded_async(comm: *mut qk_comm, d_ids: *const *const u32, n: *const usize, threshold: u32,
                                       root: c_int, streams: *const *mut c_void) -> c_int;
    pub fn qk_u64_encode_sharded_async(comm: *mut qk_comm, d_ids: *const *const u64, n: *const usize, threshold: u32,
                                       root: c_int, streams: *const *mut c_void) -> c_int;
    pub fn qk_u32_encode_sharded_wait(comm: *mut qk_comm, q: *mut qk_u32) -> c_int;
    pub fn qk_u64_encode_sharded_wait(comm: *mut qk_comm, q: *mut qk_u64) -> c_int;
    pub fn qk_u32_encode_sharded(comm: *mut qk_comm, d_ids: *const *const u32, n: *const usize, q: *mut qk_u32,
                                 root: c_int, streams: *const *mut c_void) -> c_int;
    pub fn qk_u64_encode_sharded(comm: *mut qk_comm, d_ids: *const *const u64, n: *const usize, q: *mut qk_u64,
                                 root: c_int, streams: *const *mut c_void) -> c_int;
    pub fn qk_u32_decode_sharded(comm: *mut qk_comm, diff: *const qk_u32, root: c_int, d_log: *const *const u32,
                                 n: *const usize, stop_at_last: c_int, hits: *mut u64, cap: usize,
                                 n_hits: *mut usize, streams: *const *mut c_void) -> c_int;
    pub fn qk_u64_decode_sharded(comm: *mut qk_comm, diff: *const qk_u64, root: c_int, d_log: *const *const u64,
                                 n: *const usize, stop_at_last: c_int, hits: *mut u64, cap: usize,
                                 n_hits: *mut usize, streams: *const *mut c_void) -> c_int;

    // synthetic identifier streams
    pub fn qk_fill_splitmix_u32(ctx: *mut qk_ctx, d_out: *mut u32, n: usize, seed: u64, start: u64,
                                stream: *mut c_void) -> c_int;
    pub fn qk_fill_splitmix_u64(ctx: *mut qk_ctx, d_out: *mut u64, n: usize, seed: u64, start: u64,
                                stream: *mut c_void) -> c_int;
}
