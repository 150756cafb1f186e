/*
 * Drop-in for the binary I/Q functions of SrcDsp's dsptl_files.h
 * (saveBinarySamples :101-109, readBinarySamples :250-262), plus device
 * variants that stream a capture straight into / out of HBM through pinned
 * chunks (libsrcdsp_hip.so).  readBinarySamples clears the output first and
 * returns whole samples only: the reference calls out.empty() (a no-op) and
 * appends one indeterminate sample at EOF -- both fixed.
 */
#ifndef SRCDSP_DROPIN_DSPTL_FILES_H
#define SRCDSP_DROPIN_DSPTL_FILES_H

#include <fstream>
#include <iterator>

#include "srcdsp_dropin_common.h"

namespace dsptl {

/// dsptl_files.h:101-109
template <class Type>
void saveBinarySamples(std::vector<std::complex<Type>> &in, std::ofstream &os) {
    static_assert(sizeof(std::complex<Type>) == 2 * sizeof(Type), "");
    os.write(reinterpret_cast<char *>(in.data()), in.size() * sizeof(std::complex<Type>));
    os.flush();
}

/// dsptl_files.h:250-262 (fixed: cleared output, whole samples only)
template <class Type>
void readBinarySamples(std::ifstream &is, std::vector<std::complex<Type>> &out) {
    out.clear();
    Type iq[2];
    while (is.read(reinterpret_cast<char *>(iq), sizeof(iq))) out.push_back(std::complex<Type>(iq[0], iq[1]));
}

/// device-resident capture -> file (D2H overlapped with fwrite)
template <class Type>
void saveBinarySamples(const DeviceSpan<const std::complex<Type>> &in, const char *path, bool append = false,
                       void *stream = nullptr) {
    srcdsp_detail::check(srcdsp_iq_save(path, in.data, in.size, sizeof(Type), append ? 1 : 0, stream),
                         "saveBinarySamples(device)");
}

/// file -> device memory (fread overlapped with H2D); returns the sample count
template <class Type>
size_t readBinarySamples(const char *path, DeviceSpan<std::complex<Type>> out, void *stream = nullptr) {
    size_t n = 0;
    srcdsp_detail::check(srcdsp_iq_load(path, sizeof(Type), out.data, out.size, &n, stream),
                         "readBinarySamples(device)");
    return n;
}

/// number of whole samples in a capture (to size the device buffer)
template <class Type>
size_t countBinarySamples(const char *path) {
    size_t n = 0;
    srcdsp_detail::check(srcdsp_iq_count(path, sizeof(Type), &n), "countBinarySamples");
    return n;
}

}  // namespace dsptl
#endif
