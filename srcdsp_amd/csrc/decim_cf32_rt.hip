// decim_cf32_rt.hip -- the complex<float> headline kernel with the tap count
// at run time (any N <= kCfMaxTaps; dnsampling_filters.h:136 and
// filters.h:90 take any length).
#include "cf32_launch.h"

namespace srcdsp {

// the runtime-tap headline kernel at any M it is built for
int launch_cf32_rt(DecimLaunch L, int channels, unsigned M, bool fma, hipStream_t s) {
    switch (M) {
    case 1: return launch_cf32<0, 1>(L, channels, fma, s);
    case 2: return launch_cf32<0, 2>(L, channels, fma, s);
    case 3: return launch_cf32<0, 3>(L, channels, fma, s);
    case 4: return launch_cf32<0, 4>(L, channels, fma, s);
    case 6: return launch_cf32<0, 6>(L, channels, fma, s);
    case 8: return launch_cf32<0, 8>(L, channels, fma, s);
    case 12: return launch_cf32<0, 12>(L, channels, fma, s);
    default: return launch_cf32<0, 16>(L, channels, fma, s);
    }
}

}  // namespace srcdsp
