// ia_imgwin.h — the window of one 128-row stage of an image-form DB (ia_internal.h ImgDb),
// shared by the screen (ia_screen16.hip, expanded into the MFMA operand) and the exact
// stage (ia_match.hip, re-screened row by row in fp32).
//
// A stage is 128 pixels x0 .. x0 + 127 of scanline y of one A' image.  Its window holds,
// as 16-B pieces of split pairs (hi | lo << 16, one u32 per pixel):
//   fine   rows y-2..y+2 of A, then y-2..y of A'   8 rows x WF_PC pieces (136 px from x0-4)
//   coarse rows y/2-1..y/2+1 of A, then of A'      6 rows x WC_PC pieces (72 px from x0/2-4)
//   the stage's 128 norm slots                      32 pieces
// 412 pieces, 6592 B.  Feature k of the stage's pixel p sits at byte win_off(k) + 4 p (fine
// features and the norm slot) or win_off(k) + 4 (p / 2) (coarse features).
#pragma once
#include "ia_internal.h"

namespace ia {

constexpr int WF_PC = 34, WC_PC = 18;                                 // 16-B pieces per window row
constexpr int WB_FINE = 8 * WF_PC * 16, WB_COARSE = 6 * WC_PC * 16, WB_NORM = 128 * 4;
constexpr int WIN_B = WB_FINE + WB_COARSE + WB_NORM;                  // 6592 B
constexpr int WIN_PIECES = WIN_B / 16;                                // 412

// byte offset of feature k's hi half in the window minus its lane term (pixel p of the stage:
// 4 p for fine features, 4 (p / 2) for coarse ones); lo halves are 2 bytes on
__host__ __device__ constexpr int win_off(int k) {
    return k < 9 ? WB_FINE + (k / 3) * WC_PC * 16 + (k % 3 + 3) * 4
         : k < 34 ? ((k - 9) / 5) * WF_PC * 16 + ((k - 9) % 5 + 2) * 4
         : k < 43 ? WB_FINE + (3 + (k - 34) / 3) * WC_PC * 16 + ((k - 34) % 3 + 3) * 4
         : k < 55 ? (5 + (k - 43) / 5) * WF_PC * 16 + ((k - 43) % 5 + 2) * 4
         : WB_FINE + WB_COARSE;
}
__host__ __device__ constexpr bool win_coarse(int k) { return k < 9 || (k >= 34 && k < 43); }

// where a stage's window comes from: its A' image and the pixel (y, x0) of local row lrow
// (a multiple of 128: the stage never crosses a scanline since W % 128 == 0)
struct WinSrc {
    const uint32_t *fp, *cp;   // the A' image's fine and coarse sections
    int y, x0;
    long lrow;
};
__device__ __forceinline__ WinSrc win_src(const ImgDb &im, long lrow) {
    const unsigned g = (unsigned)(im.row0 + lrow);   // < 2^31 (img_db_applies)
    const unsigned img = g / (unsigned)im.hw;
    const unsigned rem = g - img * (unsigned)im.hw;
    WinSrc w;
    w.y = (int)(rem / (unsigned)im.W);
    w.x0 = (int)(rem - (unsigned)w.y * (unsigned)im.W);
    w.fp = im.ap + img * im.apstride;
    w.cp = w.fp + im.apc;
    w.lrow = lrow;
    return w;
}
// the source of the window's 16-B piece i (< WIN_PIECES); padded rows = image rows + IMG_PY
__device__ __forceinline__ const uint32_t *win_piece(const ImgDb &im, const WinSrc &w, int i) {
    if (i < 8 * WF_PC) {
        const int r = i / WF_PC, pc = i - r * WF_PC;
        return (r < 5 ? im.fa + (long)(w.y + r) * im.Wp : w.fp + (long)(w.y + r - 5) * im.Wp) + w.x0 + 4 * pc;
    }
    if (i < 8 * WF_PC + 6 * WC_PC) {
        const int q = i - 8 * WF_PC, r = q / WC_PC, pc = q - r * WC_PC;
        return (r < 3 ? im.ca + (long)((w.y >> 1) + 1 + r) * im.Wcp
                      : w.cp + (long)((w.y >> 1) + r - 2) * im.Wcp) + (w.x0 >> 1) + 4 * pc;
    }
    return im.norm + w.lrow + 4 * (i - 8 * WF_PC - 6 * WC_PC);
}

}  // namespace ia
