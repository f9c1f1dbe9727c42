/*
 * fks_shapec.cpp — the compiler process of the robot-shape specialisation (fks_specialize.cpp).
 *
 *   fks_shapec <out.hsaco> <hiprtc option>...
 *
 * Compiles the kernel source this program carries (fks_spec_sources.inc: fks_kernels.hip and
 * the headers it includes, exactly the files libfks_hip.so was built from) with hiprtc and the
 * given options (--offload-arch, -O3, -ffp-contract=off, -DFKS_SHAPE_*), and writes the code
 * object.  It runs as a child process of the library so that the compiler is always the one
 * of the ROCm installation the library was built against: inside a process that loaded
 * PyTorch, the hiprtc and comgr PyTorch bundles (an older ROCm) would be used instead and
 * allocate registers differently.  Exit status 0 on success; the compiler log on stderr.
 * A host program only (no GPU use).
 */
#include <hip/hiprtc.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "fks_spec_sources.inc"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <out.hsaco> <hiprtc option>...\n", argv[0]);
        return 2;
    }
    const char* main_name = nullptr;
    std::string main_src;
    std::vector<std::string> hdr_src;
    std::vector<const char*> hdr_ptr, hdr_name;
    for (int i = 0; i < kFksEmbeddedSourceCount; ++i) {
        const auto& src = kFksEmbeddedSources[i];
        std::string text(reinterpret_cast<const char*>(src.data), src.size);
        if (std::strcmp(src.name, "fks_kernels.hip") == 0) {
            main_name = src.name;
            main_src = std::move(text);
        } else {
            hdr_src.push_back(std::move(text));
            hdr_name.push_back(src.name);
        }
    }
    for (const auto& t : hdr_src) hdr_ptr.push_back(t.c_str());
    if (!main_name) {
        std::fprintf(stderr, "fks_shapec carries no kernel source\n");
        return 1;
    }
    hiprtcProgram prog = nullptr;
    hiprtcResult r = hiprtcCreateProgram(&prog, main_src.c_str(), main_name, (int)hdr_ptr.size(), hdr_ptr.data(), hdr_name.data());
    if (r != HIPRTC_SUCCESS) {
        std::fprintf(stderr, "hiprtcCreateProgram: %s\n", hiprtcGetErrorString(r));
        return 1;
    }
    std::vector<const char*> opts(argv + 2, argv + argc);
    r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    if (r != HIPRTC_SUCCESS) {
        size_t n = 0;
        if (hiprtcGetProgramLogSize(prog, &n) == HIPRTC_SUCCESS && n > 1) {
            std::string log(n, '\0');
            (void)hiprtcGetProgramLog(prog, &log[0]);
            std::fprintf(stderr, "%s\n", log.c_str());
        }
        std::fprintf(stderr, "hiprtcCompileProgram: %s\n", hiprtcGetErrorString(r));
        (void)hiprtcDestroyProgram(&prog);
        return 1;
    }
    size_t n = 0;
    if (hiprtcGetCodeSize(prog, &n) != HIPRTC_SUCCESS || n == 0) {
        std::fprintf(stderr, "hiprtcGetCodeSize failed\n");
        return 1;
    }
    std::vector<char> code(n);
    r = hiprtcGetCode(prog, code.data());
    (void)hiprtcDestroyProgram(&prog);
    if (r != HIPRTC_SUCCESS) {
        std::fprintf(stderr, "hiprtcGetCode: %s\n", hiprtcGetErrorString(r));
        return 1;
    }
    FILE* f = std::fopen(argv[1], "wb");
    if (!f) {
        std::fprintf(stderr, "cannot write %s\n", argv[1]);
        return 1;
    }
    const bool ok = std::fwrite(code.data(), 1, n, f) == n;
    return (std::fclose(f) == 0 && ok) ? 0 : 1;
}
