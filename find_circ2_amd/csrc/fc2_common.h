// Internal helpers shared by the HIP and host translation units of libfc2.so.
#pragma once
#include <stdint.h>
#include <string>

#include "../../include/fc2_bp.h"

// 1 only in A/B builds (libfc2_ab.so, `make ab`): fc2_set_tuning and the measured-and-rejected kernel
// forms it selects (64-bit words, persistent grid, 256/1024-pair staged blocks, cached streaming).
#ifndef FC2_AB_FORMS
#define FC2_AB_FORMS 0
#endif

namespace fc2 {

// Thread-local message behind fc2_last_error().
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

// Largest internal length l handled by the register kernel (NW = 8 words of
// 64 positions hold l + 2 <= 512 window bases).
constexpr int kMaxFastL = 510;

// Validate the options the hot path reads; returns FC2_OK or FC2_E_PARAM.
int validate_params(const fc2_params *p);

// fc2_reorder.hip tuning (fc2_set_tuning)
extern int g_reorder_rounds;
extern int g_reorder_nt;
extern int g_reorder_shift;

inline int eff_anchor(const fc2_params *p) { return p->asize - p->margin; }  // find_circ.py:882

}  // namespace fc2
