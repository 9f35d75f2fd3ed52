// Differential / sanitizer driver for the native PGM header parser (gol_engine.cpp,
// parse_pgm_header: gol/io.go:97-117 rules).  Built only by `make -C gol-distributed-final_amd/csrc
// asan` with AddressSanitizer + UndefinedBehaviorSanitizer (host code; no GPU call is made) and run
// by tests/test_sanitizers_cpu.py, which compares every verdict with golhip.pgm.pgm_header.
//
// stdin: records of  int64 W, int64 H, uint32 n, n header bytes.
// stdout: one line per record: "<rc> <offset>" (offset -1 on error).
#include "../../gol-distributed-final_amd/csrc/gol_engine.cpp"

#include <cstdio>

int main()
{
    int64_t wh[2];
    uint32_t n;
    std::vector<uint8_t> buf;
    while (fread(wh, sizeof wh, 1, stdin) == 1 && fread(&n, sizeof n, 1, stdin) == 1) {
        buf.assign(n, 0);
        if (n && fread(buf.data(), 1, n, stdin) != n) return 2;
        // an exact-size heap copy, so a read past the header is an ASan report
        uint8_t *h = new uint8_t[n ? n : 1];
        memcpy(h, buf.data(), n);
        int64_t off = -1;
        const int rc = parse_pgm_header(h, n, wh[0], wh[1], &off);
        delete[] h;
        printf("%d %lld\n", rc, (long long)(rc == GOL_OK ? off : -1));
    }
    return 0;
}
