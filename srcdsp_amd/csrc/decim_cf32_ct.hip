// decim_cf32_ct.hip -- the complex<float> headline kernel with the tap count
// compiled in (FilterDnsamplingFir / FilterFir, dnsampling_filters.h:129-172,
// filters.h:131-169): the BASELINE lengths and their power-of-two neighbours.
#include "cf32_launch.h"

namespace srcdsp {

// the headline kernel with the tap count compiled in, where it is
// (SRCDSP_ERR_UNSUPPORTED otherwise: the caller takes the runtime-tap kernel)
int launch_cf32_compiled(DecimLaunch L, int channels, unsigned M, int N, bool fma, hipStream_t s) {
#define SRCDSP_CF(NT_, M_) \
    if (M == M_ && N == NT_) return launch_cf32<NT_, M_>(L, channels, fma, s)
    SRCDSP_CF(127, 4); SRCDSP_CF(128, 4); SRCDSP_CF(63, 4); SRCDSP_CF(64, 4);
    SRCDSP_CF(127, 8); SRCDSP_CF(128, 8); SRCDSP_CF(255, 8); SRCDSP_CF(256, 8);
    SRCDSP_CF(127, 16); SRCDSP_CF(128, 16); SRCDSP_CF(255, 16); SRCDSP_CF(256, 16);
    SRCDSP_CF(63, 2); SRCDSP_CF(64, 2); SRCDSP_CF(127, 2); SRCDSP_CF(128, 2);
    SRCDSP_CF(63, 3); SRCDSP_CF(64, 3); SRCDSP_CF(127, 3); SRCDSP_CF(128, 3);
    SRCDSP_CF(63, 1); SRCDSP_CF(64, 1);
#undef SRCDSP_CF
    return SRCDSP_ERR_UNSUPPORTED;
}

}  // namespace srcdsp
