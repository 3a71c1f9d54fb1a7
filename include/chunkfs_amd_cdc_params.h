/*
 * chunkfs_amd_cdc_params.h -- constants of the Rabin / UltraCDC / LeapCDC /
 * SeqCDC chunkers (reference src/chunkers/{rabin,ultra,leap,seq}.rs), shared
 * by the HIP engine and the CPU oracle the way chunkfs_amd_tables.h is.
 *
 * PARITY UNPINNED.  The reference takes these algorithms from the crate
 * cdc-chunkers 0.1.3 (Cargo.lock:143-151), whose source is not in this
 * environment.  The constants below follow the published
 * algorithm descriptions (DESIGN.md "Rabin, UltraCDC, LeapCDC, SeqCDC"); a
 * maintainer pins parity by replacing them with the crate's values.
 */
#ifndef CHUNKFS_AMD_CDC_PARAMS_H
#define CHUNKFS_AMD_CDC_PARAMS_H
#include <stdint.h>

/* Rabin: fingerprint over a sliding window of CDC_RABIN_WINDOW bytes modulo
 * an irreducible polynomial of degree 53 (table-driven append / slide-out);
 * cut where (digest & (2^round(log2 avg) - 1)) == 0. */
#define CDC_RABIN_POLY 0x3DA3358B4DC173ULL
#define CDC_RABIN_WINDOW 48u

/* UltraCDC: Hamming distance of the last 8 bytes to the pattern 0xAA..AA,
 * tested against MASK_S before the normal size and MASK_L after it; low-
 * entropy strings (LEST repeats of an identical 8-byte block) cut early. */
#define CDC_ULTRA_PATTERN 0xAAu
#define CDC_ULTRA_MASK_S 0x2Fu
#define CDC_ULTRA_MASK_L 0x2Cu
#define CDC_ULTRA_LEST 64u

/* LeapCDC: a cut after position p needs 24 consecutive eligible windows
 * ending at p, p-1, ..., p-23 (22 primary, then 2 secondary), each window
 * CDC_LEAP_WSIZE bytes; a failing window at distance k leaps the candidate
 * forward by 24 - k.  That leap structure follows the Leap-based CDC paper.
 *
 * STAND-IN ELIGIBILITY FUNCTION.  The window test below -- a table hash of
 * the window (CDC_LEAP_SEED) compared with a threshold chosen so that 24
 * successes have probability ~2^-bits, bits = round(log2(avg - min)) -- is
 * this build's own placeholder, NOT the published Leap-based CDC eligibility
 * function (which cdc-chunkers 0.1.3 builds from random draws: it depends on
 * rand 0.8.5 / rand_distr 0.4.3, Cargo.lock:143-151, absent here).  The
 * chunker is therefore "Leap-shaped", not LeapCDC.  Pinning means replacing
 * the eligibility function (bits_kernel's primary / secondary predicates and
 * oracle cut_leap); every constant it uses is one named value here. */
#define CDC_LEAP_WINDOWS 24u
#define CDC_LEAP_PRIMARY 22u
#define CDC_LEAP_WSIZE 5u
#define CDC_LEAP_SEED 0x1EA9CDC5EEDULL
/* floor(2^32 * 2^(-bits/24)), bits = 0..32 (saturated at 2^32 - 1). */
static const uint32_t CDC_LEAP_THRESHOLD[33] = {
    0xFFFFFFFFu, /*  0 */
    0xF8B6513Au, /*  1 */
    0xF1A1BF38u, /*  2 */
    0xEAC0C6E7u, /*  3 */
    0xE411F03Au, /*  4 */
    0xDD93CDD7u, /*  5 */
    0xD744FCCAu, /*  6 */
    0xD124243Eu, /*  7 */
    0xCB2FF529u, /*  8 */
    0xC5672A11u, /*  9 */
    0xBFC886BBu, /* 10 */
    0xBA52D7EFu, /* 11 */
    0xB504F333u, /* 12 */
    0xAFDDB68Fu, /* 13 */
    0xAADC0847u, /* 14 */
    0xA5FED6A9u, /* 15 */
    0xA14517CCu, /* 16 */
    0x9CADC958u, /* 17 */
    0x9837F051u, /* 18 */
    0x93E298E0u, /* 19 */
    0x8FACD61Eu, /* 20 */
    0x8B95C1E3u, /* 21 */
    0x879C7C96u, /* 22 */
    0x83C02CFAu, /* 23 */
    0x80000000u, /* 24 */
    0x7C5B289Du, /* 25 */
    0x78D0DF9Cu, /* 26 */
    0x75606373u, /* 27 */
    0x7208F81Du, /* 28 */
    0x6EC9E6EBu, /* 29 */
    0x6BA27E65u, /* 30 */
    0x6892121Fu, /* 31 */
    0x6597FA94u, /* 32 */};

/* SeqCDC: a cut after SEQ_LENGTH consecutive byte pairs in the operation
 * mode's direction (increasing: b[i] > b[i-1]); after JUMP_TRIGGER opposing
 * pairs the scan jumps JUMP_SIZE bytes ahead.  Defaults of seq::Config. */
#define CDC_SEQ_LENGTH 5u
#define CDC_SEQ_JUMP_TRIGGER 50u
#define CDC_SEQ_JUMP_SIZE 256u

/* round(log2(x)) in integers (x >= 1), shared so host and oracle agree. */
static inline uint32_t cdc_log2_round(uint64_t x)
{
    uint32_t b = 63u - (uint32_t)__builtin_clzll(x);
    if (b > 0 && b < 63 && x - (1ull << b) >= (1ull << b) / 2) ++b;
    return b;
}

#endif
