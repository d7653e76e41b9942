// philox.hpp -- Philox4x32-10 counter RNG and the integer-only overlay model,
// shared by host and device code of libgossip_hip (compiled by hipcc only).
//
// Replaces the reference's std::random_device -> mt19937 (peer.cpp:215-216)
// so that a run is a pure function of (rng_seed, peer, purpose, counter):
// the same draw on the CPU and on every GPU of a partition.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gossip {

// Counter purpose words (ctr[0]); key = {rng_seed, peer}.  DESIGN.md section 3.
enum : uint32_t {
    P_DEGREE = 1,   // {1, response, 0, 0}.x        k draw            (peer.cpp:220-222)
    P_TARGET = 2,   // {2, response, i>>2, 0}[i&3]  candidate i       (powerlaw list)
    P_SHUFFLE = 3,  // {3, response, d>>2, 0}[d&3]  Fisher-Yates draw (peer.cpp:224-225)
    P_CHURN = 4,    // key {seed, v >> 2}, {4, round, 0, 0}[v & 3]: death test of peer v (one draw per 4 peers)
    P_ORIGIN = 5,   // key {seed, ~0u}, {5, k, attempt, 0}.x  origin pick
    P_REBOOT = 6,   // {6, round, dead, 0}.x k draw; {6, round, dead, 1+(i>>2)}[i&3] candidate i (re-bootstrap)
    P_REJOIN = 7,   // {7, round, 0, 0}.x restart test, .y k draw; {7, round, 1+(i>>2), 0}[i&3] candidate i
};

struct u32x4 {
    uint32_t x, y, z, w;
};

__host__ __device__ inline u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                               uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return u32x4{c0, c1, c2, c3};
}

__host__ __device__ inline uint32_t lane_of(const u32x4& r, uint32_t i) {
    return i == 0 ? r.x : i == 1 ? r.y : i == 2 ? r.z : r.w;
}

// c = floor(n * V^3), V = x / 2^32, by truncated 64-bit products: Chung-Lu
// weights ~ c^(-2/3) -> degree power law with exponent 2.5 (alpha, peer.cpp:219).
__host__ __device__ inline uint32_t skew_pick(uint32_t x, uint64_t n) {
    const uint64_t a = ((uint64_t)x * x) >> 32;
    const uint64_t b = (a * x) >> 32;
    return (uint32_t)((n * b) >> 32);
}

// Digest weight g(i): splitmix64 finaliser of i+1, forced odd.  The round
// digest is sum_i g(i) * seen_word[i] mod 2^64 -- a function of the seen set
// only, so it can be accumulated from the fresh words of each round.
__host__ __device__ inline uint64_t digest_weight(uint64_t idx) {
    uint64_t z = (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z | 1ull;
}

}  // namespace gossip
