/*
 * fks_shapec.cpp — the compiler process of the robot-shape specialisation (fks_specialize.cpp).
 *
 *   fks_shapec <out.hsaco> <source dir> <hiprtc option>...
 *
 * Compiles <source dir>/fks_kernels.hip with the headers beside it (the library writes there
 * the sources it carries: fks_kernels.hip and the headers it includes, exactly the files
 * libfks_hip.so was built from) with hiprtc and the given options (--offload-arch, -O3,
 * -ffp-contract=off, -DFKS_SHAPE_*), and writes the code object.  It runs as a child process
 * of the library so that the compiler is always the one of the ROCm installation the library
 * was built against: inside a process that loaded PyTorch, the hiprtc and comgr PyTorch
 * bundles (an older ROCm) would be used instead and allocate registers differently.  Exit
 * status 0 on success; the compiler log on stderr.  A host program only (no GPU use).
 */
#include <hip/hiprtc.h>

#include <cstdio>
#include <filesystem>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

namespace {

bool slurp(const std::filesystem::path& p, std::string* out) {
    std::ifstream f(p, std::ios::binary);
    if (!f) return false;
    out->assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <out.hsaco> <source dir> <hiprtc option>...\n", argv[0]);
        return 2;
    }
    const std::filesystem::path dir(argv[2]);
    std::string main_src;
    if (!slurp(dir / "fks_kernels.hip", &main_src)) {
        std::fprintf(stderr, "no fks_kernels.hip in %s\n", argv[2]);
        return 1;
    }
    std::vector<std::string> hdr_src, hdr_name;
    std::error_code ec;
    for (const auto& e : std::filesystem::directory_iterator(dir, ec)) {
        const std::string name = e.path().filename().string();
        if (!e.is_regular_file() || name == "fks_kernels.hip") continue;
        std::string text;
        if (!slurp(e.path(), &text)) {
            std::fprintf(stderr, "cannot read %s\n", e.path().c_str());
            return 1;
        }
        hdr_src.push_back(std::move(text));
        hdr_name.push_back(name);
    }
    std::vector<const char*> hdr_ptr, hdr_nptr;
    for (size_t i = 0; i < hdr_src.size(); ++i) {
        hdr_ptr.push_back(hdr_src[i].c_str());
        hdr_nptr.push_back(hdr_name[i].c_str());
    }
    hiprtcProgram prog = nullptr;
    hiprtcResult r = hiprtcCreateProgram(&prog, main_src.c_str(), "fks_kernels.hip", (int)hdr_ptr.size(), hdr_ptr.data(), hdr_nptr.data());
    if (r != HIPRTC_SUCCESS) {
        std::fprintf(stderr, "hiprtcCreateProgram: %s\n", hiprtcGetErrorString(r));
        return 1;
    }
    std::vector<const char*> opts(argv + 3, argv + argc);
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
