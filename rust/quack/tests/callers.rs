//! The reference callers' use of the crate, restated as tests (needs the
//! `strawmen` feature, as both callers enable it).  The host paths run
//! anywhere libquack_hip.so loads; the device test needs a gfx950 GPU and
//! returns early without one.
#![cfg(feature = "strawmen")]

use quack::arithmetic::{self, ModularArithmetic};
use quack::{Context, PowerSumQuack, PowerSumQuackU32, PowerSumQuackU64, StrawmanAQuack, StrawmanBQuack};
use std::collections::VecDeque;

fn ids(n: usize, seed: u32) -> Vec<u32> {
    (0..n as u32).map(|i| (i ^ seed).wrapping_mul(2_654_435_761).rotate_left(7)).collect()
}

/// sidekick.rs:32,42,48,187,203: build, insert per packet, reset, snapshot, serialize.
#[test]
fn sidekick_sender_side() {
    let threshold = 10;
    let mut quack = PowerSumQuackU32::new(threshold);
    for id in ids(1000, 1) {
        quack.insert(id);
    }
    assert_eq!(quack.count(), 1000);
    let snapshot = quack.clone();
    let bytes = bincode::serialize(&snapshot).unwrap();
    let back: PowerSumQuackU32 = bincode::deserialize(&bytes).unwrap();
    assert_eq!(back, quack);
    quack = PowerSumQuackU32::new(threshold);
    assert_eq!(quack.count(), 0);
    assert_eq!(quack.last_value(), None);
}

/// media_client.rs:216-319: the receiver's decode round.
#[test]
fn media_client_decode_round() {
    let threshold = 20;
    let log = ids(5000, 2);
    let lost: Vec<usize> = vec![10, 999, 2500, 4998];
    let mut sender = PowerSumQuackU32::new(threshold);
    for (i, &id) in log.iter().enumerate() {
        if !lost.contains(&i) {
            sender.insert(id);
        }
    }
    // the proxy's quACK arrives serialized
    let quack: PowerSumQuackU32 = bincode::deserialize(&bincode::serialize(&sender).unwrap()).unwrap();
    let mut my_quack = PowerSumQuackU32::new(threshold);
    let mut last_index = 0;
    for (i, &id) in log.iter().enumerate() {
        my_quack.insert(id);
        if Some(id) == quack.last_value() {
            last_index = i;
            break;
        }
    }
    let reset1 = my_quack.count() < quack.count();
    let reset2 = my_quack.count() > quack.count() + threshold as u32;
    assert!(!reset1 && !reset2);
    let mut diff_quack = my_quack.clone();
    diff_quack.sub_assign(quack);
    let coeffs = diff_quack.to_coeffs();
    let mut missing = Vec::new();
    for &id in &log[..=last_index] {
        if Some(id) == diff_quack.last_value() {
            break;
        }
        if arithmetic::eval(&coeffs, id).value() == 0 {
            missing.push(id);
        }
    }
    let want: Vec<u32> = lost.iter().filter(|&&i| i < last_index).map(|&i| log[i]).collect();
    assert_eq!(missing, want);
    for id in &missing {
        my_quack.remove(*id);
    }
}

/// sender_strawman_{a,b}.rs + media_client.rs:173,191: plain serde structs.
#[test]
fn strawmen_round_trip() {
    let a = StrawmanAQuack { sidekick_id: 0xDEAD_BEEF };
    let b: StrawmanAQuack = bincode::deserialize(&bincode::serialize(&a).unwrap()).unwrap();
    assert_eq!(a, b);
    let w = StrawmanBQuack { window: VecDeque::from(vec![1, 2, 3]), window_size: 8 };
    let v: StrawmanBQuack = bincode::deserialize(&bincode::serialize(&w).unwrap()).unwrap();
    assert_eq!(w, v);
}

/// fig2_microbenchmarks.py:226-227: the u64 sketch over GF(2^64 - 59).
#[test]
fn u64_decode() {
    let log: Vec<u64> = (0..300u64).map(|i| i.wrapping_mul(0x9E37_79B9_7F4A_7C15)).collect();
    let mut a = PowerSumQuackU64::new(10);
    let mut b = PowerSumQuackU64::new(10);
    for (i, &x) in log.iter().enumerate() {
        a.insert(x);
        if i % 37 != 5 {
            b.insert(x);
        }
    }
    a.sub_assign(b);
    let got = a.decode_with_log(&log);
    let want: Vec<u64> = log.iter().enumerate().filter(|(i, _)| i % 37 == 5).map(|(_, &x)| x).collect();
    assert_eq!(got, want);
}

/// The batch path from host memory (qk_u32_encode_host): equal to per-id inserts.
#[test]
fn batch_insert_on_the_gpu() {
    let n = match Context::device_count() {
        Ok(n) => n,
        Err(_) => return,
    };
    if n == 0 {
        return;
    }
    let ctx = Context::new(0).unwrap();
    let stream = ids(1 << 20, 3);
    let mut gpu = PowerSumQuackU32::new(32);
    gpu.insert_batch(&ctx, &stream).unwrap();
    let mut cpu = PowerSumQuackU32::new(32);
    for &id in &stream {
        cpu.insert(id);
    }
    assert_eq!(gpu, cpu);
}
