// wo_jitc: compiles one generated specialised-kernel source with the system ROCm's
// hiprtc, in a process of its own.  The library runs it (trace_kernels.hip
// jit_compile) when the hiprtc serving the library's process is another ROCm's -- a
// process that imported torch first runs on torch's bundled HIP runtime, hiprtc and
// comgr, whose older compiler spills where the system's does not (DESIGN.md §0 round 6
// item 2).  Links only hiprtc (no GPU is touched).
//
//   wo_jitc <source file> <code object out> [hiprtc options ...]   exit 0: compiled
#include <hip/hiprtc.h>

#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "jit_sources.inc"

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: wo_jitc <source> <out> [options...]\n");
        return 2;
    }
    std::string src;
    {
        FILE* f = fopen(argv[1], "rb");
        if (!f) return 3;
        char buf[65536];
        size_t n;
        while ((n = fread(buf, 1, sizeof buf, f)) > 0) src.append(buf, n);
        fclose(f);
    }
    const char* hdr_src[] = {kEmbed_wo_device_common_h, kEmbed_wo_scene_h};
    const char* hdr_names[] = {"wo_device_common.h", "wololo/wo_scene.h"};
    hiprtcProgram p;
    if (hiprtcCreateProgram(&p, src.c_str(), "wo_scene_jit.hip", 2, hdr_src, hdr_names) != HIPRTC_SUCCESS) return 4;
    std::vector<const char*> opts(argv + 3, argv + argc);
    if (hiprtcCompileProgram(p, (int)opts.size(), opts.data()) != HIPRTC_SUCCESS) {
        size_t ls = 0;
        hiprtcGetProgramLogSize(p, &ls);
        std::string log(ls + 1, '\0');
        hiprtcGetProgramLog(p, &log[0]);
        fprintf(stderr, "%.2000s\n", log.c_str());
        hiprtcDestroyProgram(&p);
        return 5;
    }
    size_t cs = 0;
    hiprtcGetCodeSize(p, &cs);
    std::vector<char> code(cs);
    hiprtcGetCode(p, code.data());
    hiprtcDestroyProgram(&p);
    FILE* o = fopen(argv[2], "wb");
    if (!o) return 6;
    const bool ok = fwrite(code.data(), 1, code.size(), o) == code.size();
    return fclose(o) == 0 && ok ? 0 : 7;
}
