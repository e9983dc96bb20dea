// decode_file: one zd_decompress of a file (host in / host out), for chasing
// a failure outside Python: prints the status and the output length, and on
// SIGABRT / SIGSEGV the native backtrace (addresses resolve with addr2line
// against the same libzd.so).
//   decode_file <input.zst> [flags [output file]]
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <vector>

#include "zd.h"

static void on_signal(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  char msg[64];
  const int m = snprintf(msg, sizeof msg, "decode_file: signal %d, backtrace:\n", sig);
  (void)!write(2, msg, (size_t)m);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <input.zst> [flags]\n", argv[0]);
    return 2;
  }
  signal(SIGABRT, on_signal);
  signal(SIGSEGV, on_signal);
  FILE* f = fopen(argv[1], "rb");
  if (!f) { perror(argv[1]); return 2; }
  std::vector<uint8_t> src;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) src.insert(src.end(), buf, buf + k);
  fclose(f);
  const uint32_t flags = argc > 2 ? (uint32_t)strtoul(argv[2], nullptr, 0) : 0u;
  zd_plan* P = nullptr;
  int st = zd_plan_create(src.data(), src.size(), flags, &P);
  if (st) { printf("plan_create %d\n", st); return 1; }
  zd_plan_info info{};
  zd_plan_info_get(P, &info);
  zd_plan_destroy(P);
  size_t cap = info.out_bytes ? info.out_bytes : 1, out_len = 0;
  for (int pass = 0; pass < 2; pass++) {
    std::vector<uint8_t> out(cap);
    st = zd_decompress(src.data(), src.size(), out.data(), cap, &out_len, flags);
    printf("pass %d: status %d, out_len %zu (cap %zu)\n", pass, st, out_len, cap);
    fflush(stdout);
    if (out_len <= cap) break;
    cap = out_len;
  }
  // the same through a kept plan: where the first failing frame stopped
  std::vector<uint8_t> out(cap);
  if (zd_plan_create(src.data(), src.size(), flags, &P) == 0) {
    st = zd_plan_decompress(P, src.data(), src.size(), out.data(), cap, &out_len);
    zd_plan_info_get(P, &info);
    if (argc > 3) {
      FILE* o = fopen(argv[3], "wb");
      if (o) { fwrite(out.data(), 1, out_len < cap ? out_len : cap, o); fclose(o); }
    }
    const unsigned long long k = info.error_key;
    if (k == ~0ull)
      printf("plan: status %d, replans %llu\n", st, (unsigned long long)info.replans);
    else
      printf("plan: status %d, replans %llu, key phase %llu block %llu stage %llu sub %llu\n", st,
             (unsigned long long)info.replans, k >> 62, (k >> 32) & 0x3FFFFFFF, (k >> 28) & 15, (k >> 8) & 0xFFFFF);
    zd_plan_destroy(P);
  }
  return 0;
}
