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

// 24-bit multiplies: full-rate VALU ops on gfx950 (v_mul_u32_u24 /
// v_mul_hi_u32_u24), where a 32-bit v_mul_lo_u32 is a multi-pass op.  The
// compiler selects them from these exact forms; the host computes the same.
__host__ __device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t b) {
    return (a & 0xffffffu) * (b & 0xffffffu);
}
__host__ __device__ __forceinline__ uint32_t mulhi24(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)(a & 0xffffffu) * (uint64_t)(b & 0xffffffu)) >> 32);
}

// Prefix Bloom filter for keys of 3..7 bytes.  A key lives in ONE 32-bit word
// chosen by its first three bytes (so every length >= 3 of a window position
// shares the word: one LDS read per position) and sets ONE bit of it, chosen
// from bytes the key owns by a length-specific 24-bit multiply.  With
// lo = bytes 0..3 and hi = bytes 4..7 of the window (little-endian):
//   word   = mul24(lo, kPfWord) >> (32 - wlog)             bytes 0..2
//   bit(3) = mulhi24(lo, C3)                               bytes 0..2
//   bit(4) = mulhi24(lo >> 8, C4)                          bytes 1..3
//   bit(5) = mulhi24(lo >> 16 | hi << 16, C5)              bytes 2..4
//   bit(6) = mulhi24(lo >> 24 | hi << 8, C6)               bytes 3..5
//   bit(7) = mulhi24(x, C7) ^ mulhi24(x >> 8, C7b), x = lo >> 24 | hi << 8   bytes 3..6
// (each mod 32).  No form reads a byte at or past klen, so the bytes after a
// window never need masking.
constexpr uint32_t kPfWord = 0x9E3779u;
constexpr uint32_t kPfC3 = 0x7F4A7Du, kPfC4 = 0x58F1B5u, kPfC5 = 0xC2B2AFu, kPfC6 = 0x27D4EBu, kPfC7 = 0x165667u,
                   kPfC7b = 0xD3A2E5u;

__host__ __device__ __forceinline__ uint32_t pf_word(uint32_t lo, uint32_t shift) { return mul24(lo, kPfWord) >> shift; }

// bit position (low 5 bits significant) of a key of klen (3..7) bytes
__host__ __device__ __forceinline__ uint32_t pf_bit(int klen, uint32_t lo, uint32_t hi) {
    switch (klen) {
        case 3: return mulhi24(lo, kPfC3);
        case 4: return mulhi24(lo >> 8, kPfC4);
        case 5: return mulhi24((lo >> 16) | (hi << 16), kPfC5);
        case 6: return mulhi24((lo >> 24) | (hi << 8), kPfC6);
        default: {
            const uint32_t x = (lo >> 24) | (hi << 8);
            return mulhi24(x, kPfC7) ^ mulhi24(x >> 8, kPfC7b);
        }
    }
}

// Filter image (host-built, staged whole into LDS): a direct 256-bit bitmap
// of the 1-byte keys, a direct 65536-bit bitmap of the 2-byte keys, then the
// prefix Bloom words.
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
