// Offline hiprtc compile of a dumped specialised source (KINHIP_JIT_DUMP, rebuilt against the current
// device headers by tools/jit_offline.py) with the options kinhip_jit.cpp uses; writes the code object
// for register / spill inspection (llvm-readelf --notes).  No GPU needed.
//   hipcc -O2 tools/jit_rtc_check.cpp -o /tmp/jit_rtc_check -lhiprtc
//   /tmp/jit_rtc_check src.hip out.co [-DNAME=VALUE ...]
#include <hip/hiprtc.h>

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s src.hip out.co [-Dopt ...]\n", argv[0]);
        return 2;
    }
    std::ifstream in(argv[1]);
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string src = ss.str();
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "kinhip_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) return 1;
    std::vector<const char*> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize", "-DKINHIP_JIT=1",
                                     "-DKINHIP_IK_NARROW=1"};
    for (int i = 3; i < argc; ++i) opts.push_back(argv[i]);
    const hiprtcResult r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    if (ls > 1) {
        std::string log(ls, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        fprintf(stderr, "%s\n", log.c_str());
    }
    if (r != HIPRTC_SUCCESS) return 1;
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    std::vector<char> code(n);
    hiprtcGetCode(prog, code.data());
    std::ofstream(argv[2], std::ios::binary).write(code.data(), (std::streamsize)n);
    return 0;
}
