// lsmck_diag.h -- the segment walk's A/B knobs and clock marks, for
// diagnostic builds only: tools/build_ab.sh builds (EXTRA="-DLSMCK_DIAG
// -DLSMCK_LATER_MIN=..." and the like), tools/segwalk_repairs.py's host
// models, and -DLSMCK_SEG_CLOCK builds (tools/seg_clock.py).  The product
// build never includes it: lsmck_segwalk.h then fixes the values below.
#ifndef LSMCK_DIAG_H
#define LSMCK_DIAG_H
#include <stdint.h>

// per-segment clock marks: lsmck_wal.hip defines the real one (before this
// header) in -DLSMCK_SEG_CLOCK builds; every other unit gets none
#ifndef LSMCK_SEG_CLOCK_MARK
#define LSMCK_SEG_CLOCK_MARK(k, slot)
#endif
#ifndef LSMCK_LATER_SKIP_TO
#define LSMCK_LATER_SKIP_TO 131072
#endif
#ifndef LSMCK_LATER_MIN
#define LSMCK_LATER_MIN 65536
#endif
#ifndef LSMCK_LATER_SCAN
#define LSMCK_LATER_SCAN 65536
#endif
#ifndef LSMCK_SCAN_BLOCKS
#define LSMCK_SCAN_BLOCKS 1
#endif

namespace lsmck {
namespace seg {
namespace tune {
constexpr uint64_t kLaterSkipTo = LSMCK_LATER_SKIP_TO;
constexpr uint64_t kLaterMin = LSMCK_LATER_MIN;
constexpr uint64_t kLaterScan = LSMCK_LATER_SCAN;
constexpr int kScanBlocks = LSMCK_SCAN_BLOCKS;
#ifdef LSMCK_SEG_LATER_ALWAYS  // (host model A/B, tools/segwalk_repairs.py: the later-start rule everywhere)
constexpr bool kLaterAlways = true;
#else
constexpr bool kLaterAlways = false;
#endif
}  // namespace tune
}  // namespace seg
}  // namespace lsmck
#endif
