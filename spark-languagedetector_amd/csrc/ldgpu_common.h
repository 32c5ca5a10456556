// ldgpu_common.h -- shared by the HIP kernels and the host runtime of libldgpu.so.
//
// Gram key format (device and host): a window of klen <= 7 bytes b0..b(klen-1)
// packs into one u64
//     key = b0 | b1 << 8 | ... | b(klen-1) << 8(klen-1) | klen << 56
// so equality of keys == structural equality of the reference's Seq[Byte]
// keys (LanguageDetector.scala:26, LanguageDetectorModel.scala:132), including
// the length (a partial window "ab" of a 2-byte document at n=3 IS the 2-gram
// "ab").  key 0 never occurs (klen >= 1) and marks an empty hash slot.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ldgpu {

constexpr int kMaxGram = 7;
constexpr int kMaxLangs = 256;
constexpr int kMaxGramLengths = 32;
constexpr uint64_t kEmpty = 0;

// Filter hash -- cheap: 32-bit multiplies only, and for klen <= 4 the high
// word is the constant klen << 24 so its product is wave-uniform.
__host__ __device__ __forceinline__ uint32_t hi_mix(uint32_t hi) { return hi * 0x85EBCA77u; }
__host__ __device__ __forceinline__ uint32_t filter_hash(uint32_t lo, uint32_t himix) {
    return (lo * 0x9E3779B1u) ^ himix;
}
__host__ __device__ __forceinline__ uint32_t filter_hash_key(uint64_t key) {
    return filter_hash((uint32_t)key, hi_mix((uint32_t)(key >> 32)));
}

// Blocked Bloom filter for keys of 3..7 bytes: a key sets / tests TWO bits of
// ONE 32-bit word, so a probe is one LDS read and one multiply.  word = top
// `wlog` bits of h; the two bit positions are the 10 bits below them.
__host__ __device__ __forceinline__ uint32_t filter_bits(uint32_t h, uint32_t shift) {
    return (1u << ((h >> (shift - 5)) & 31u)) | (1u << ((h >> (shift - 10)) & 31u));
}

// Filter image (host-built, staged whole into LDS): a direct 256-bit bitmap
// of the 1-byte keys, a direct 65536-bit bitmap of the 2-byte keys, then the
// blocked Bloom words.
constexpr uint32_t kBmp1Words = 8;
constexpr uint32_t kBmp2Words = 2048;
constexpr uint32_t kBloomBase = kBmp1Words + kBmp2Words;

// Candidate queue entry: klen in the top 3 bits, window position below.
constexpr uint32_t kPosBits = 29;
constexpr int64_t kMaxDocBytes = (int64_t)1 << kPosBits;

// Slot hash for the device hash tables (splitmix64 finaliser).
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t k) {
    k ^= k >> 31;
    k *= 0x7fb5d329728ea185ull;
    k ^= k >> 27;
    k *= 0x81dadef4bc2dd44dull;
    k ^= k >> 33;
    return k;
}

__host__ __device__ __forceinline__ int key_len(uint64_t key) { return (int)(key >> 56); }

inline uint64_t pack_key_host(const uint8_t* p, int len) {
    uint64_t k = (uint64_t)len << 56;
    for (int i = 0; i < len; ++i) k |= (uint64_t)p[i] << (8 * i);
    return k;
}

// (length, unsigned bytes) order of a packed key: length in the top byte,
// the bytes big-endian below it (the build's top-K tie-break).
__host__ __device__ __forceinline__ uint64_t sort_key(uint64_t key) {
    const int len = key_len(key);
    uint64_t s = (uint64_t)len << 56;
    for (int i = 0; i < len; ++i) s |= ((key >> (8 * i)) & 0xffull) << (48 - 8 * i);
    return s;
}

// Number of windows of Scala sliding(n) over len bytes (partial rule).
__host__ __device__ __forceinline__ int64_t n_windows(int64_t len, int n) {
    return len == 0 ? 0 : (len < n ? 1 : len - n + 1);
}

// Slot of the SCORE hash table (32 B = two dwordx4 loads): key, row index
// (bit 31 set = row of the wrong length, LDGPU_EROWLEN on hit) and, for
// mask-form tables, the row's value and its first 64-language mask word, so a
// hit needs no further dependent load when L <= 64.
struct alignas(16) Slot {
    uint64_t key;
    uint32_t row;
    uint32_t pad;
    double val;
    uint64_t mask0;
};

constexpr uint32_t kBadRow = 0x80000000u;

}  // namespace ldgpu
