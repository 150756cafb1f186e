/*
 * Drop-in for SrcDsp's mixers.h: dsptl::Mixer<complex<int16_t>,
 * complex<int16_t>, int16_t, N> (reference mixers.h:27-188, the only
 * specialisation the reference defines), executed by libsrcdsp_hip.so.
 */
#ifndef SRCDSP_DROPIN_MIXERS_H
#define SRCDSP_DROPIN_MIXERS_H

#include "srcdsp_dropin_common.h"

namespace dsptl {

template <class InType, class OutType, class PhaseType, unsigned N = 4096>
class Mixer;  // primary template declared, not defined (mixers.h:120-121)

template <unsigned N>
class Mixer<std::complex<int16_t>, std::complex<int16_t>, int16_t, N> {
public:
    /// mixers.h:149-159 + _Mixer(): phi = freq = 0
    Mixer() : h_(nullptr) { srcdsp_detail::check(srcdsp_mixer_create(&h_, N), "Mixer"); }
    ~Mixer() { srcdsp_mixer_destroy(h_); }
    /// copies (mixers.h:27-48 / 134-160 are value types): table, phi, freq
    Mixer(const Mixer &o) : h_(srcdsp_detail::clone_handle(o.h_, srcdsp_mixer_clone, "Mixer(copy)")) {}
    Mixer(Mixer &&o) noexcept : h_(o.h_) { o.h_ = nullptr; }
    Mixer &operator=(Mixer o) noexcept {
        std::swap(h_, o.h_);
        return *this;
    }

    /// mixers.h:51-67
    void setFrequency(float loFreq) {
        assert(loFreq <= 1 && loFreq >= -1);
        srcdsp_detail::check(srcdsp_mixer_set_frequency(h_, loFreq), "setFrequency");
    }
    /// mixers.h:76-81
    void reset(float loFreq = 0) { srcdsp_detail::check(srcdsp_mixer_reset(h_, loFreq), "reset"); }
    /// mixers.h:91-98
    void adjustFrequency(float loFreq = 0) {
        srcdsp_detail::check(srcdsp_mixer_adjust_frequency(h_, loFreq), "adjustFrequency");
    }
    /// mixers.h:169-188 (non-const input, as the reference)
    void step(std::vector<std::complex<int16_t>> &in, std::vector<std::complex<int16_t>> &out) {
        srcdsp_detail::check_size(out.size() >= in.size(), "Mixer::step");
        srcdsp_detail::check(srcdsp_mixer_step_host(h_, in.data(), in.size(), out.data()), "Mixer::step");
    }
    void step(const DeviceSpan<const std::complex<int16_t>> &in, DeviceSpan<std::complex<int16_t>> out,
              void *stream = nullptr) {
        srcdsp_detail::check_size(out.size >= in.size, "Mixer::step(device)");
        srcdsp_detail::check(srcdsp_mixer_step(h_, in.data, in.size, out.data, stream), "Mixer::step(device)");
    }
    srcdsp_mixer_t handle() const { return h_; }

private:
    srcdsp_mixer_t h_;
};

}  // namespace dsptl
#endif
