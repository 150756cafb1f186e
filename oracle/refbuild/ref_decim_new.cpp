// Reference-build harness TU: dsptl_dnsampling_filters.h (current header).
// Same canonical include order as ref_decim_old.cpp.
#include <cmath>
#include <cassert>
#include <complex>
#include <cstdint>
#include <vector>
#include <array>
#include "dsptl_dnsampling_filters.h"
#include "ref_api.h"
#define REF_HAS_SETCOEFFS 1
#include "ref_decim_box.inc"

extern "C" {
void *ref_decim2_create(int variant, unsigned M, const void *coeffs, int ntaps) {
    return makeDecim(variant, M, coeffs, ntaps);
}
void ref_decim2_set_coeffs(void *h, const void *coeffs, int ntaps) {
    static_cast<DecimBase *>(h)->setCoeffs(coeffs, ntaps);
}
void ref_decim2_set_left_shift(void *h, int ls) { static_cast<DecimBase *>(h)->leftShift(ls); }
void ref_decim2_reset(void *h) { static_cast<DecimBase *>(h)->reset(); }
void ref_decim2_step(void *h, const void *in, long n_in, void *out) {
    static_cast<DecimBase *>(h)->step(in, n_in, out);
}
void ref_decim2_destroy(void *h) { delete static_cast<DecimBase *>(h); }
}
