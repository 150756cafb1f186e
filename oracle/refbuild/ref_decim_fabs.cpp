// Reference-build harness TU pinning the OTHER abs() binding: <math.h> (the
// libstdc++ wrapper, which brings std::abs(float) into :: ) is included first, so
// dnsampling_filters.h:94 computes sum(fabs(c)) instead of sum(abs((int)c)).
#include <math.h>
#include <cmath>
#include <cassert>
#include <complex>
#include <cstdint>
#include <vector>
#include <array>
#include "dnsampling_filters.h"
#include "ref_api.h"
#define REF_FLOAT_ONLY 1
#include "ref_decim_box.inc"

extern "C" {
void *ref_decim_fabs_create(int variant, unsigned M, const void *coeffs, int ntaps) {
    return makeDecim(variant, M, coeffs, ntaps);
}
void ref_decim_fabs_step(void *h, const void *in, long n_in, void *out) {
    static_cast<DecimBase *>(h)->step(in, n_in, out);
}
void ref_decim_fabs_destroy(void *h) { delete static_cast<DecimBase *>(h); }
}
