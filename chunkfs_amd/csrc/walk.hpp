// walk.hpp -- the segment-walk engine for Rabin / UltraCDC / LeapCDC / SeqCDC
// (reference src/chunkers/{rabin,ultra,leap,seq}.rs; DESIGN.md "Segment walk").
//
// Every stream of the batch is cut into segments of 2^seg_log2 bytes (a chunk
// may span whole segments: they then hold no start, E = X).  One wave (bitmap
// mode; one lane in byte mode) owns one segment and runs the
// algorithm's exact byte-serial cut rule (the same rule as oracle/cdc_oracle.c)
// from a warm-up start `warm` bytes before the segment, recording the chunk
// starts that fall inside it.  A chain from the warm-up start usually merges
// with the true chain before the segment starts; the fix-up rounds re-walk
// every segment whose entry differs from its predecessor's exit (Jacobi), and
// a serial pass finishes whatever is left, so the result is exact whether or
// not the chains merge.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cdc_kernels.hpp"

namespace cdc {
namespace walk {

// Verdict of one fix-up round from its flag block: ch = chains whose exit
// changed, q = those of them whose changed exit was a quiet-run re-walk.
// Settled: nothing changed.  Quiet: mostly quiet runs -- chains there keep
// their phase and each round moves the true one a single segment, so the
// in-order pass takes over.  One rule for the host's round loop
// (Engine::run_walk), the device's round gate (round_stops) and the gated
// output after the first group (emit_skips).
enum : int { kRoundSettled = 0, kRoundQuiet = 1, kRoundGoOn = 2 };
__host__ __device__ __forceinline__ int round_verdict(unsigned long long ch, unsigned long long q) {
    return ch == 0 ? kRoundSettled : (2 * q >= ch ? kRoundQuiet : kRoundGoOn);
}
// Rounds in the first group of fix-up launches, behind which the output is
// queued and gated on the device (Engine::run_walk; emit_skips).
constexpr unsigned kFirstGroupRounds = 1;

struct WalkParams {
    uint32_t algo;            // cdc_algo_t: 2 rabin, 4 ultra, 5 leap, 6 seq
    uint32_t min, avg, max;
    uint64_t rabin_mask;      // (1 << round(log2 avg)) - 1
    uint32_t rabin_shift;     // deg(poly) - 8
    uint32_t leap_thr;        // eligibility threshold (CDC_LEAP_THRESHOLD)
    uint32_t seq_mode, seq_len, seq_trig, seq_jump;
    uint32_t cap;             // chunk starts recorded per segment
    uint64_t warm;            // warm-up bytes before a segment
    const uint64_t *tabs;     // device [768]: rabin mod[256], rabin out[256], leap hash[256]
    // Bitmap mode (Rabin with min >= 48, Ultra, Leap): the per-position
    // predicates of bits_kernel, nbm bitmaps interleaved per 64-bit word:
    // word k of bitmap b of segment g at bm[(g * seg_words + k) * nbm + b].
    uint64_t *bm;
    uint32_t nbm;             // 0 = byte mode; Rabin 1 (hit), Ultra 3 (mask_s, mask_l, 8-byte repeat), Leap 2
    uint32_t seg_words;       // 64-bit words per segment and bitmap (segment bytes / 64)
    uint32_t piece_log2;      // the data-parallel passes run over pieces of 2^piece_log2 bytes (<= segment)
    uint32_t bits_fine;       // bitmap pass: lane per 64-position word (Ultra, Leap, Seq)
    uint32_t ahead;           // fix-up round: segments one lane may re-walk (1 = plain Jacobi)
    uint32_t wave;            // 1: wave-cooperative walk_kernel (Rabin / UltraCDC bitmap mode)
    // Link mode (LeapCDC): the rule's candidate cut positions (content-defined:
    // every cut that is not a max / end cut lands on one) are listed per
    // segment, and the next chunk start after a chunk starting at each of
    // them is computed once, a lane per candidate (link_kernel); the walks
    // then hop over links and walk the rule only from other starts.  A
    // segment with more than ccap candidates (low-entropy data) keeps direct
    // walks.
    uint32_t links;           // 1: link mode
    uint32_t ccap;            // candidates per segment
    uint32_t *ccnt;           // [S] candidates of each segment (> ccap: overflowed, no links)
    uint32_t *cpos;           // [S * ccap] their segment offsets, ascending
    uint64_t *lnext;          // [S * ccap] next chunk start (stream offset) after a chunk starting there
    uint32_t *lidx;           // [S * ccap] candidate slot of that next start, kVirt | v, or kNoCand
    // Virtual starts: a link's next start that is not a candidate (a max cut)
    // gets its own link (vnext / vidx), so that a walk never walks the rule
    // from a start a link reached; up to kVirtRounds levels deep.
    uint32_t vcap;            // virtual entries (8 per segment; past it: kNoCand, the walk walks)
    unsigned long long *vcnt; // [2 * kVirtRounds + 2]: entries allocated, per round: first entry of the round
    uint64_t *vpos;           // [vcap] stream offset of the virtual start
    uint32_t *vseg;           // [vcap] its stream's first segment (for find_cand)
    uint64_t *vnext;          // [vcap] next start after a chunk starting there
    uint32_t *vidx;           // [vcap] slot of that next start (candidate, kVirt | v, kNoCand)
    // LeapCDC wave walks: per 64-position word w, the leap orbit of each
    // entry candidate 64 w + e (e < 24) through the word, jt[w * 24 + e]:
    // < 24 = its entry into word w + 1, >= 64 = accepted at 64 w + (v - 64).
    uint8_t *jt;
    // ... and per 512-position block b (8 words) the same through the whole
    // block, jt8[b * 24 + e] (u16): < 24 = entry into block b + 1, >= 512 =
    // accepted at 512 b + (v - 512).
    uint16_t *jt8;
    // Wave walks: one "quiet" bit per bitmap word, bit k & 63 of rsum[k >> 6]
    // (k = segment g's word index + g * seg_words), written by the bitmap
    // pass: Rabin no hit, SeqCDC no in-direction pair, UltraCDC all 8-byte
    // repeats, LeapCDC all windows eligible.  Chains inside long quiet runs
    // (zero-filled or constant regions), where every chunk has one fixed
    // length, take the run's chunks many at a time (walk.hip quiet_run).
    // nullptr when the bitmap pass in use does not write it
    // (bits_write_summary).
    uint64_t *rsum;
    // ... and per segment, bit k: every summary word of quiet kind k is all
    // quiet (a stream's last segment: 0), from qseg_kernel after the bitmap
    // pass.  A fix-up round lets one chain cross a stretch of such segments
    // whole (walk.hip serial_run); nullptr with rsum.
    uint8_t *qseg;
};

constexpr uint32_t kNoCand = 0xFFFFFFFFu;
constexpr uint32_t kVirt = 0x80000000u;
constexpr uint32_t kVirtRounds = 3;

struct WalkState {
    uint64_t *E;      // [S] entry: first chunk start >= segment start
    uint64_t *X;      // [S] exit: first chunk start >= segment end (or the stream length)
    uint32_t *N;      // [S] chunk starts inside the segment
    uint64_t *list;   // [S * cap] those starts (stream offsets)
    uint64_t *Xs;     // [S] exits snapshot of a fix-up round
    uint64_t *Es;     // [S] entries snapshot of a fix-up round
    uint64_t *P;      // [S + 1] exclusive prefix of N (chunk index of each segment)
    uint64_t *bsum;   // [blocks + 1] per-block sums of the prefix
    uint64_t *first;  // [n + 1] chunk index of each stream's first chunk
    unsigned long long *flags;  // [4]: 0 exits changed this round, 1 errors, 2 lowest such segment, 3 re-walks
    // Fix-up round only: the previous round's flag block; the round returns at
    // once when that round changed no exit (null: always run).
    const unsigned long long *gate;
};

constexpr uint32_t kMaxFixRounds = 16;  // flag blocks allocated after the main one

constexpr int kScanBlock = 256;  // prefix / emit block (segments per block)

// Bitmap mode: the predicate bitmaps of every segment (wave per segment).
// Whether the bitmap pass launch_bits picks for wp writes the quiet-run
// summary (wp.rsum may be non-null only then).
bool bits_write_summary(const WalkParams &wp);
hipError_t launch_bits(const StreamTable &st, const WalkParams &wp, hipStream_t s);
// Zeroes the main flag block and the `rounds` round blocks after it (their
// word 2, the lowest changed segment, to ~0): one launch instead of three fills.
hipError_t launch_flags_init(unsigned long long *flags, uint32_t rounds, hipStream_t s);
// Link mode: candidate lists (wave per segment), then the links (lane per candidate).
hipError_t launch_links(const StreamTable &st, const WalkParams &wp, hipStream_t s);
hipError_t launch_walk(const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s);
// One Jacobi round: snapshot X and E (one launch; snap = false for round 0,
// whose snapshot the walk itself wrote), then re-walk every segment whose
// entry is not its predecessor's exit, stopping where the new chain meets the
// old one.  flags[0] counts the re-walks that changed an exit (the host loops
// while > 0).
hipError_t launch_fix(const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s,
                      bool snap = true);
// Exact in-order pass over all segments from the lowest one re-walked.
hipError_t launch_serial(const StreamTable &st, const WalkParams &wp, const WalkState &ws, hipStream_t s);
// Prefix of N, first[], and the Chunk{offset,length} output.  egate (the
// first of egate_rounds round flag blocks) non-null: every kernel returns at
// once unless those rounds settled (the host's rule, run_walk), so the output
// can be queued behind the first group of rounds without a host round trip.
hipError_t launch_emit(const StreamTable &st, const WalkParams &wp, const WalkState &ws, void *d_out,
                       uint64_t out_cap, hipStream_t s, const unsigned long long *egate = nullptr,
                       uint32_t egate_rounds = 0);
// The same output behind the first group (egate, egate_rounds) in two
// launches: finish_kernel (one block: the prefix of N as P[], first[] into
// the workspace and into h_first, the go word for the gated emit, the flag
// blocks of `rounds` rounds into h_flags, and -- when the output is due -- the
// flags reset for the next call), then emit_kernel.  h_first / h_flags are
// host-coherent pinned memory.  For batches of <= 2^16 segments (finish_fits).
bool finish_fits(const StreamTable &st);
hipError_t launch_finish_emit(const StreamTable &st, const WalkParams &wp, const WalkState &ws, void *d_out,
                              uint64_t out_cap, hipStream_t s, const unsigned long long *egate,
                              uint32_t egate_rounds, uint32_t rounds, uint64_t *go, uint64_t *h_first,
                              uint64_t *h_flags);

}  // namespace walk
}  // namespace cdc
