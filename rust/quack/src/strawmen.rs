//! The strawman "quACKs" the sidekick senders serialize instead of a power-sum
//! sketch (feature `strawmen`, enabled by both callers:
//! `sidekick/Cargo.toml:9`, `media_integration/media/Cargo.toml:11`).
//! Plain serde structs — no arithmetic, nothing on the GPU.

use serde::{Deserialize, Serialize};
use std::collections::VecDeque;

/// Strawman 1a: echo the identifier of every packet
/// (`sender_strawman_a.rs:54-56`, `sender_strawman_tcp.rs:65-67`,
/// `media_client.rs:173`).
#[derive(Clone, Debug, PartialEq, Eq, Serialize, Deserialize)]
pub struct StrawmanAQuack {
    pub sidekick_id: u32,
}

/// Strawman 1b: echo a sliding window of the last identifiers
/// (`sender_strawman_b.rs:57-64`, `media_client.rs:191`).
#[derive(Clone, Debug, PartialEq, Eq, Serialize, Deserialize)]
pub struct StrawmanBQuack {
    pub window: VecDeque<u32>,
    pub window_size: usize,
}
