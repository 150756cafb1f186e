// Reference-build harness TU: dnsampling_filters.h (obsolete header, 127 taps legal).
// Canonical oracle recipe: <cmath>,<cassert>,<complex>,<cstdint>,
// <vector>,<array> first, NO <math.h>/<stdlib.h>, so abs(float) binds to ::abs(int).
#include <cmath>
#include <cassert>
#include <complex>
#include <cstdint>
#include <vector>
#include <array>
#include "dnsampling_filters.h"
#include "ref_api.h"
#include "ref_decim_box.inc"

extern "C" {
void *ref_decim_create(int variant, unsigned M, const void *coeffs, int ntaps) {
    return makeDecim(variant, M, coeffs, ntaps);
}
void ref_decim_set_left_shift(void *h, int ls) { static_cast<DecimBase *>(h)->leftShift(ls); }
void ref_decim_reset(void *h) { static_cast<DecimBase *>(h)->reset(); }
void ref_decim_step(void *h, const void *in, long n_in, void *out) {
    static_cast<DecimBase *>(h)->step(in, n_in, out);
}
void ref_decim_destroy(void *h) { delete static_cast<DecimBase *>(h); }
/* step() timed around the reference call alone (excludes the harness copies);
 * used by bench.py's cpu_baseline leg */
double ref_decim_step_timed(void *h, const void *in, long n_in, void *out) {
    return static_cast<DecimBase *>(h)->stepTimed(in, n_in, out);
}
}
