// Layout of the RLC partial (cc_rlc_partial_device -> all-gather -> cc_rlc_finish_device, SURVEY.md
// §8e), 32-bit words:
//   [0, 144)                        the shard's Miller product (Fp12, Montgomery words in slot order)
//   [144]                           its fall-back flag (an identity or non-subgroup sigma, a bad verkey)
//   RLC_WIN_OFF + RLC_WIN_WORDS w   the shard's fold window sum S_w (fold.hip), w < 16: 48 words affine
//                                   (G2: x.a x.b y.a y.b; G1: x y, then zeros), then its identity flag
// The window pairs e(S_w, (256^w) g~) are evaluated once per batch in the finish (over every shard's
// windows), not in the partial: there they would add one wave slot's worth of loops to a Miller launch
// that exactly fills the chip (2,048 waves at config 3).
#pragma once

constexpr int RLC_F12_WORDS = 144;
constexpr int RLC_FLAG = 144;
constexpr int RLC_WINDOWS = 16;
constexpr int RLC_WIN_OFF = 145;
constexpr int RLC_WIN_WORDS = 49;
constexpr int RLC_PART_WORDS = RLC_WIN_OFF + RLC_WINDOWS * RLC_WIN_WORDS;  // 929
