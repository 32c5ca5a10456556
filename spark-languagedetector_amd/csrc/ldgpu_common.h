// ldgpu_common.h -- shared by the HIP kernels and the host runtime of libldgpu.so.
//
// Gram key format (device and host): a window of klen <= 7 bytes b0..b(klen-1)
// packs into one u64
//     key = b0 | b1 << 8 | ... | b(klen-1) << 8(klen-1) | klen << 56
// so equality of keys == structural equality of the reference's Seq[Byte]
// keys (LanguageDetector.scala:26, LanguageDetectorModel.scala:132), including
// the length (a partial window "ab" of a 2-byte document at n=3 IS the 2-gram
// "ab").  key 0 never occurs (klen >= 1) and marks an empty hash slot.
//
// Wide keys (klen 8..kMaxWideGram): two u64 words,
//     lo = b0 .. b7 (little-endian),  hi = b8 .. b(klen-1) | klen << 56
// in a table of their own (SCORE: WideSlot, whose filter bits use the first
// seven bytes and the length, as a 7-byte key's do; FIT: wide_count_kernel).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ldgpu {

constexpr int kMaxGram = 7;       // one-word keys
constexpr int kMaxWideGram = 15;  // two-word keys up to this length (SCORE tables, FIT counts)
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
// by a length-specific 24-bit multiply of three bytes the key owns.  With
// lo = bytes 0..3 and hi = bytes 4..7 of the window (little-endian):
//   word   = mul24(lo, kPfWord) >> (32 - wlog)                       bytes 0..2
//   bit(n) = mulhi24(alignbit(hi, lo, pf_shift(n)), pf_mult(n)) mod 32
// pf_shift(n) = 8 min(n - 3, 3): bytes n-3..n-1 for n <= 6, bytes 3..5 for
// n = 7.  No form reads a byte at or past n, so the bytes after a window never
// need masking, and every length runs the same two instructions.
constexpr uint32_t kPfWord = 0x9E3779u;

// per-length bit multiplier (24 bits; a scalar op on the device)
__host__ __device__ __forceinline__ constexpr uint32_t pf_mult(int klen) {
    return ((uint32_t)klen * 0x6F4F2Bu + 0x7F4A7Du) & 0xFFFFFFu;
}

__host__ __device__ __forceinline__ uint32_t pf_word(uint32_t lo, uint32_t shift) { return mul24(lo, kPfWord) >> shift; }

__host__ __device__ __forceinline__ constexpr uint32_t pf_shift(int klen) { return 8u * (uint32_t)(klen < 6 ? klen - 3 : 3); }

// bit position (low 5 bits significant) from a length's (shift, multiplier)
// (shift < 32: one v_alignbit_b32 on the device)
__host__ __device__ __forceinline__ uint32_t pf_bit_c(uint32_t lo, uint32_t hi, uint32_t shift, uint32_t c) {
    return mulhi24((uint32_t)(((((uint64_t)hi) << 32) | lo) >> shift), c);
}

__host__ __device__ __forceinline__ uint32_t pf_bit(int klen, uint32_t lo, uint32_t hi) {
    return pf_bit_c(lo, hi, pf_shift(klen), pf_mult(klen));
}

// Bits per key of the prefix Bloom (LDGPU_BLOOM_BITS, 1 or 2).  With two, a
// key sets a second bit of its word, from a second multiplier over the same
// three bytes, and a window is a candidate only when both bits are set: at
// ~2.5 keys per word the false candidates fall ~4x (every false candidate is
// an L2 verify) for two more VALU ops per test.  Measured on config 2 (same
// box, tools/ab.sh): 5.47 ms with two bits against 5.34 ms with one -- the
// verify of a 256-B document's candidates is one 64-lane batch either way, so
// the VALU cost outweighs the fewer candidates.  One bit it is.
#ifndef LDGPU_BLOOM_BITS
#define LDGPU_BLOOM_BITS 1
#endif
__host__ __device__ __forceinline__ constexpr uint32_t pf_mult2_of(uint32_t m) {
    return ((m ^ 0xA5A5A5u) * 0x2Fu + 0x1B873Du) & 0xFFFFFFu;
}
__host__ __device__ __forceinline__ uint32_t pf_bit2(int klen, uint32_t lo, uint32_t hi) {
    return pf_bit_c(lo, hi, pf_shift(klen), pf_mult2_of(pf_mult(klen)));
}

// Keyed bloom (tables whose bloom exceeds LDS): for a key of klen >= 3 bytes
// (lo / hi = its bytes, masked to klen) word = h >> (32 - wlog), bit =
// (h >> (27 - wlog)) mod 32 of h = kb_hash -- three 24-bit multiplies over
// bytes 0..2, 3..5 and (6, length), whose top bits depend on every input bit.
__host__ __device__ __forceinline__ uint32_t kb_hash(uint32_t lo, uint32_t hi, uint32_t klen) {
    const uint32_t a = lo & 0xffffffu;
    const uint32_t b = (lo >> 24) | (hi << 8);
    const uint32_t c = (hi >> 16) | (klen << 8);
    return mul24(a, 0x9E3779u) ^ mul24(b, 0x85EBCAu) ^ mul24(c ^ (a >> 12), 0xC2B2AFu);
}

// Keyed bloom, line layout (blooms beyond kKbLineBytes, ldgpu_internal.h):
// every key of >= 4 bytes of one window position -- the lengths 4..15 that
// start there -- sets its bit in ONE 64-B line (16 words) chosen by the
// position's first four bytes, so one position's tests of every length >= 4
// read one line of L2 / HBM instead of one line per length: word = line << 4
// | h >> 28, bit = (h >> 23) mod 32 of h = kb_hash, line = kb_line(bytes
// 0..3) >> (32 - (wlog - 4)).  Keys of 3 bytes, and every key of a smaller
// keyed bloom, keep a word of their own: word = h >> (32 - wlog).
__host__ __device__ __forceinline__ uint32_t kb_line(uint32_t lo) {
    return mul24(lo, 0xB5297Au) ^ mul24(lo >> 8, 0x68E31Du);
}
// The bloom word of a key of klen >= 3 bytes with kb_hash h is
// line16 + (h >> s_word), its bit (h >> s_bit) mod 32: in the line layout a
// key of >= 4 bytes takes s_word = 28, s_bit = 23 and line16 = its position's
// line << 4; a 3-byte key, or any key outside the line layout, s_word =
// wshift (= 32 - wlog), s_bit = wshift - 5 and line16 = 0.  (Both shifts
// are wave-uniform: one formula for every lane.)
__host__ __device__ __forceinline__ uint32_t kb_sword(uint32_t klen, bool lines, uint32_t wshift) {
    return lines && klen >= 4 ? 28u : wshift;
}
__host__ __device__ __forceinline__ uint32_t kb_sbit(uint32_t klen, bool lines, uint32_t wshift) {
    return lines && klen >= 4 ? 23u : wshift - 5u;
}
__host__ __device__ __forceinline__ uint32_t kb_line16(uint32_t lo, uint32_t wshift) {
    return (kb_line(lo) >> (wshift + 4)) << 4;
}

// Keyed bloom, chunk layout (count-mode tables whose keyed bloom stays
// L2-resident, chosen at build when its false-candidate estimate is no worse):
// every key of >= 3 bytes sets TWO bits of ONE 16-B chunk chosen by the first
// three bytes of its window position -- q1 = h >> 25 and q2 = (h >> 18) mod
// 128 of h = kb_hash(key) -- so a position's tests of every length read one
// 16-B chunk (one L2 request) instead of a word per length.  chunk =
// kb_chunk(lo) >> shift (shift = 32 - log2 chunks).
__host__ __device__ __forceinline__ uint32_t kb_chunk(uint32_t lo) { return kb_line(lo & 0xffffffu); }

// Filter image (host-built, staged whole into LDS): a direct 256-bit bitmap
// of the 1-byte keys, a direct 65536-bit bitmap of the 2-byte keys, then the
// prefix Bloom words.
constexpr uint32_t kBmp1Words = 8;
constexpr uint32_t kBmp2Words = 2048;
constexpr uint32_t kBloomBase = kBmp1Words + kBmp2Words;

// The 2-byte bitmap's word of key b0 | b1 << 8 (its bit: b0 & 31).  Word
// b01 >> 5 puts a wave's consecutive letter pairs on 4 LDS banks (bank = b1
// mod 4 and b0 >> 5); LDGPU_BMP2_SWZ XORs its low 3 bits with bits 2..4 of b1,
// so the lanes of an LDS read group spread over all 32 banks by their second
// byte, while lanes of one (b0 >> 5, b1) still read one word (broadcast).
#ifndef LDGPU_BMP2_SWZ
#define LDGPU_BMP2_SWZ 0
#endif
__host__ __device__ __forceinline__ uint32_t bmp2_word(uint32_t b01) {
    const uint32_t w = (b01 >> 5) & 2047u;
    return LDGPU_BMP2_SWZ ? w ^ ((b01 >> 10) & 7u) : w;
}
// the inverse: the keys of physical word wd are (bmp2_unword(wd) << 5) | bit
__host__ __device__ __forceinline__ uint32_t bmp2_unword(uint32_t wd) {
    return LDGPU_BMP2_SWZ ? wd ^ ((wd >> 5) & 7u) : wd;
}

// Candidate queue entry: klen in the top 4 bits, window position below.
constexpr uint32_t kPosBits = 28;
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

// Cuckoo slot positions of the score table (Slot, 2 choices): two 32-bit
// hashes of 24-bit multiplies over bytes 0..2, 3..5 and (6, length) --
// full-rate VALU ops, where mix64's 64-bit multiplies are multi-pass -- whose
// top bits depend on every key bit; slot 1 = h1 >> (32 - log2 cap), slot 2 =
// h2 >> (32 - log2 cap).  (lo, hi = the key's two 32-bit halves)
__host__ __device__ __forceinline__ void slot_hash(uint32_t lo, uint32_t hi, uint32_t& h1, uint32_t& h2) {
    const uint32_t a = lo & 0xffffffu;
    const uint32_t b = (lo >> 24) | (hi << 8);
    const uint32_t c = hi >> 16;
    h1 = mul24(a, 0x9E3779u) ^ mul24(b, 0x85EBCAu) ^ mul24(c ^ (a >> 12), 0xC2B2AFu);
    h2 = mul24(b ^ (c << 8), 0x27D4EBu) ^ mul24(a, 0x165667u) ^ mul24(c ^ (b >> 12), 0xD3A265u);
}

// Cuckoo slot positions of the wide-key table: the two words folded into
// slot_hash's input
__host__ __device__ __forceinline__ void wide_hash(uint64_t lo, uint64_t hi, uint32_t& h1, uint32_t& h2) {
    const uint32_t u0 = (uint32_t)hi, u1 = (uint32_t)(hi >> 32);
    const uint32_t x0 = (uint32_t)lo ^ mul24(u0 ^ (u1 << 13), 0x5BD1E9u) ^ (u1 >> 19);
    const uint32_t x1 = (uint32_t)(lo >> 32) ^ mul24((u0 >> 12) ^ u1, 0x873593u) ^ (u0 << 7);
    slot_hash(x0, x1, h1, h2);
}

__host__ __device__ __forceinline__ int key_len(uint64_t key) { return (int)(key >> 56); }

// General keys (any length; tables with a gram length beyond kMaxWideGram):
// a 64-bit hash of the key's bytes and length (FNV-1a, then mix64), host and
// device alike; the key itself is compared byte for byte against the table's
// key arena on a hash match.
__host__ __device__ __forceinline__ uint64_t gen_hash(const uint8_t* p, int64_t len) {
    uint64_t h = 1469598103934665603ull ^ (uint64_t)len;
    for (int64_t i = 0; i < len; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return mix64(h);
}

// Long-gram prefilter of mixed tables (a gram length beyond kMaxWideGram next to
// shorter ones): two bits per key of >= 16 bytes in a bitmap of 2^lb bits,
// chosen by the key's first eight bytes (lo, hi: little-endian words) and its
// length -- a window of n >= 16 bytes whose two bits are not both set is no
// key.  32-bit arithmetic only (host and device alike).
__host__ __device__ __forceinline__ void long_bits(uint32_t lo, uint32_t hi, uint32_t n, uint32_t lb, uint32_t& b1,
                                                   uint32_t& b2) {
    uint32_t h = lo * 0x9E3779B1u + ((hi * 0x85EBCA77u) << 13 | (hi * 0x85EBCA77u) >> 19) + n * 0xC2B2AE3Du;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 13;
    b1 = h >> (32 - lb);
    b2 = (h * 0x297A2D39u) >> (32 - lb);
}

// Slot of the general key table (open addressing, linear probes): the key's
// hash, its length (0: empty slot) and its row (kBadRow: wrong length).
struct alignas(16) GenSlot {
    uint64_t h;
    uint32_t len;
    uint32_t row;
};

inline uint64_t pack_key_host(const uint8_t* p, int len) {
    uint64_t k = (uint64_t)len << 56;
    for (int i = 0; i < len; ++i) k |= (uint64_t)p[i] << (8 * i);
    return k;
}

// Host-side stand-in for a FIT gram of 8..15 bytes among one-word keys:
// kWideTag << 56 | its rank in the (length, bytes) order of the table's wide
// grams.  It sorts after every one-word key (whose top byte is <= 7), so a
// key list sorted by sort_key is in (length, bytes) order throughout.
constexpr uint64_t kWideTag = 16;

// (length, unsigned bytes) order of a packed key: length in the top byte,
// the bytes big-endian below it (the build's top-K tie-break).
__host__ __device__ __forceinline__ uint64_t sort_key(uint64_t key) {
    const int len = key_len(key);
    if (len >= (int)kWideTag) return key;
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
    uint32_t pad;   // the row's one language when it has exactly one, else 0xffffffff
    double val;
    uint64_t mask0;
};

constexpr uint32_t kBadRow = 0x80000000u;

// Slot of the wide-key table (32 B): the key's two words, row index (kBadRow
// as in Slot) and the row's one language (or 0xffffffff); values and masks
// are read from the row arrays.  lo = hi = 0 marks an empty slot.
struct alignas(16) WideSlot {
    uint64_t lo, hi;
    uint32_t row;
    uint32_t lang1;
    uint32_t pad[2];
};

// Count-mode key table of big models: 2-choice buckets of 5 slots, one 64-B
// line each -- five packed keys, five 32-bit payloads, a flags word.  A
// payload is kPayLang | the row's one language, or the row index (a row of
// several languages: its mask words); kBadRow marks a row of the wrong
// length.  A key goes to its primary bucket (bucket_index of the hash's high
// half) while it has room, else to its secondary one (of the low half), and
// then its primary bucket's overflow flag (flags bit 0) is raised -- so most
// lookups read ONE line.  Any bucket count (not a power of two): the table is
// sized for ~0.85 load, so config 5's 10M keys take 150 MB, which the
// Infinity Cache holds beside the keyed bloom (4-slot buckets of 16-B slots at
// a power-of-two count took 256 MiB).
struct alignas(64) Bucket {
    uint64_t k[5];
    uint32_t p[5];
    uint32_t flags;
};
static_assert(sizeof(Bucket) == 64, "one line per bucket");
constexpr uint32_t kBucketOverflow = 1u;
constexpr uint32_t kPayLang = 0x40000000u;

__host__ __device__ __forceinline__ uint64_t bucket_index(uint32_t h, uint64_t nb) {
    return ((uint64_t)h * nb) >> 32;
}

}  // namespace ldgpu
