//! `quack::arithmetic` — elements of GF(p) and the root-test polynomial
//! evaluation the decode loop calls (`media_client.rs:21,310`:
//! `arithmetic::eval(&coeffs, id).value() == 0`).
//!
//! p32 = 2^32 - 5 and p64 = 2^64 - 59.  Host scalar code: the
//! per-element operations here are what the caller does a handful of times per
//! quACK; every batch operation runs on the GPU through `crate::ffi`.

use serde::{Deserialize, Serialize};
use std::fmt;
use std::ops::{Add, AddAssign, Mul, MulAssign, Neg, Sub, SubAssign};

/// Identifier types with a prime field behind them (u32 and u64 only).
pub trait Field: Copy + Clone + PartialEq + Eq + fmt::Debug + fmt::Display + Default + private::Sealed {
    /// The field's prime.
    const MODULUS: Self;
    fn reduce(x: Self) -> Self;
    fn add_mod(a: Self, b: Self) -> Self;
    fn sub_mod(a: Self, b: Self) -> Self;
    fn mul_mod(a: Self, b: Self) -> Self;
    fn zero() -> Self;
    fn one() -> Self;
    fn is_zero(self) -> bool;
    /// Canonical value of the monic polynomial x^d + c1 x^(d-1) + ... + cd at x
    /// (libquack_hip's `qk_*_eval`, the same Horner step the GPU root test runs).
    fn eval_monic(coeffs: &[Self], x: Self) -> Self;
    fn to_u128(self) -> u128;
}

mod private {
    pub trait Sealed {}
    impl Sealed for u32 {}
    impl Sealed for u64 {}
}

impl Field for u32 {
    const MODULUS: u32 = crate::ffi::QK_P32;
    fn reduce(x: u32) -> u32 {
        if x >= Self::MODULUS { x - Self::MODULUS } else { x }
    }
    fn add_mod(a: u32, b: u32) -> u32 {
        ((a as u64 + b as u64) % Self::MODULUS as u64) as u32
    }
    fn sub_mod(a: u32, b: u32) -> u32 {
        ((a as u64 + Self::MODULUS as u64 - b as u64) % Self::MODULUS as u64) as u32
    }
    fn mul_mod(a: u32, b: u32) -> u32 {
        ((a as u64 * b as u64) % Self::MODULUS as u64) as u32
    }
    fn zero() -> u32 { 0 }
    fn one() -> u32 { 1 }
    fn is_zero(self) -> bool { self == 0 }
    fn eval_monic(coeffs: &[u32], x: u32) -> u32 {
        unsafe { crate::ffi::qk_u32_eval(coeffs.as_ptr(), coeffs.len() as u32, x) }
    }
    fn to_u128(self) -> u128 { self as u128 }
}

impl Field for u64 {
    const MODULUS: u64 = crate::ffi::QK_P64;
    fn reduce(x: u64) -> u64 {
        if x >= Self::MODULUS { x - Self::MODULUS } else { x }
    }
    fn add_mod(a: u64, b: u64) -> u64 {
        ((a as u128 + b as u128) % Self::MODULUS as u128) as u64
    }
    fn sub_mod(a: u64, b: u64) -> u64 {
        ((a as u128 + Self::MODULUS as u128 - b as u128) % Self::MODULUS as u128) as u64
    }
    fn mul_mod(a: u64, b: u64) -> u64 {
        ((a as u128 * b as u128) % Self::MODULUS as u128) as u64
    }
    fn zero() -> u64 { 0 }
    fn one() -> u64 { 1 }
    fn is_zero(self) -> bool { self == 0 }
    fn eval_monic(coeffs: &[u64], x: u64) -> u64 {
        unsafe { crate::ffi::qk_u64_eval(coeffs.as_ptr(), coeffs.len() as u32, x) }
    }
    fn to_u128(self) -> u128 { self as u128 }
}

/// An element of GF(p), always canonical (< p).  Serialized by serde as a
/// struct of one field, i.e. exactly its value in bincode.
#[derive(Clone, Copy, PartialEq, Eq, Hash, Default, Serialize, Deserialize)]
pub struct ModularInteger<T> {
    value: T,
}

/// The accessor trait the decode loop imports (`media_client.rs:21`).
pub trait ModularArithmetic {
    type T;
    /// `x mod p`.
    fn new(x: Self::T) -> Self;
    /// The canonical representative.
    fn value(&self) -> Self::T;
    fn zero() -> Self;
    fn is_zero(&self) -> bool;
    fn pow(&self, e: u64) -> Self;
    /// Multiplicative inverse (Fermat); the inverse of 0 is 0.
    fn inv(&self) -> Self;
}

impl<T: Field> ModularInteger<T> {
    /// Wrap a value already known to be canonical (< p).
    pub(crate) fn from_canonical(value: T) -> Self {
        debug_assert!(value.to_u128() < T::MODULUS.to_u128());
        ModularInteger { value }
    }
}

impl<T: Field> ModularArithmetic for ModularInteger<T> {
    type T = T;
    fn new(x: T) -> Self {
        ModularInteger { value: T::reduce(x) }
    }
    fn value(&self) -> T {
        self.value
    }
    fn zero() -> Self {
        ModularInteger { value: T::zero() }
    }
    fn is_zero(&self) -> bool {
        self.value.is_zero()
    }
    fn pow(&self, mut e: u64) -> Self {
        let mut base = self.value;
        let mut acc = T::one();
        while e > 0 {
            if e & 1 == 1 {
                acc = T::mul_mod(acc, base);
            }
            base = T::mul_mod(base, base);
            e >>= 1;
        }
        ModularInteger { value: acc }
    }
    fn inv(&self) -> Self {
        let e = (T::MODULUS.to_u128() - 2) as u64;
        self.pow(e)
    }
}

impl<T: Field> Add for ModularInteger<T> {
    type Output = Self;
    fn add(self, rhs: Self) -> Self {
        ModularInteger { value: T::add_mod(self.value, rhs.value) }
    }
}
impl<T: Field> AddAssign for ModularInteger<T> {
    fn add_assign(&mut self, rhs: Self) {
        self.value = T::add_mod(self.value, rhs.value);
    }
}
impl<T: Field> Sub for ModularInteger<T> {
    type Output = Self;
    fn sub(self, rhs: Self) -> Self {
        ModularInteger { value: T::sub_mod(self.value, rhs.value) }
    }
}
impl<T: Field> SubAssign for ModularInteger<T> {
    fn sub_assign(&mut self, rhs: Self) {
        self.value = T::sub_mod(self.value, rhs.value);
    }
}
impl<T: Field> Mul for ModularInteger<T> {
    type Output = Self;
    fn mul(self, rhs: Self) -> Self {
        ModularInteger { value: T::mul_mod(self.value, rhs.value) }
    }
}
impl<T: Field> MulAssign for ModularInteger<T> {
    fn mul_assign(&mut self, rhs: Self) {
        self.value = T::mul_mod(self.value, rhs.value);
    }
}
impl<T: Field> Neg for ModularInteger<T> {
    type Output = Self;
    fn neg(self) -> Self {
        ModularInteger { value: T::sub_mod(T::zero(), self.value) }
    }
}

impl<T: fmt::Debug> fmt::Debug for ModularInteger<T> {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "{:?}", self.value)
    }
}
impl<T: fmt::Display> fmt::Display for ModularInteger<T> {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "{}", self.value)
    }
}

/// The root-test polynomial at x: canonical value of
/// x^d + c1 x^(d-1) + ... + cd, d = coeffs.len(); zero iff x is congruent to
/// a missing id (`media_client.rs:310`).
pub fn eval<T: Field>(coeffs: &Vec<ModularInteger<T>>, x: T) -> ModularInteger<T> {
    let c: Vec<T> = coeffs.iter().map(|m| m.value).collect();
    ModularInteger { value: T::eval_monic(&c, x) }
}
