// zd_diag — decode a .zst file through the C ABI with a SIGSEGV backtrace
// handler (debug aid for the GPU box, where no debugger is available).
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../include/zd.h"

static void on_segv(int sig) {
  void* bt[64];
  int n = backtrace(bt, 64);
  fprintf(stderr, "signal %d, backtrace:\n", sig);
  backtrace_symbols_fd(bt, n, 2);
  _exit(139);
}

int main(int argc, char** argv) {
  signal(SIGSEGV, on_segv);
  signal(SIGBUS, on_segv);
  if (argc < 2) { fprintf(stderr, "usage: zd_diag file.zst\n"); return 2; }
  FILE* f = fopen(argv[1], "rb");
  if (!f) { perror(argv[1]); return 2; }
  std::vector<uint8_t> in;
  uint8_t buf[65536];
  size_t r;
  while ((r = fread(buf, 1, sizeof buf, f)) > 0) in.insert(in.end(), buf, buf + r);
  fclose(f);
  fprintf(stderr, "read %zu bytes\n", in.size());
  zd_plan* P = nullptr;
  int st = zd_plan_create(in.data(), in.size(), 0, &P);
  fprintf(stderr, "zd_plan_create -> %d (%s)\n", st, zd_status_name(st));
  if (st) return 1;
  zd_plan_info I;
  zd_plan_info_get(P, &I);
  fprintf(stderr, "frames %llu blocks %llu out %llu\n", (unsigned long long)I.nframes,
          (unsigned long long)I.nblocks, (unsigned long long)I.out_bytes);
  zd_plan_destroy(P);
  std::vector<uint8_t> out(I.out_bytes + 16);
  size_t ol = 0;
  st = zd_decompress(in.data(), in.size(), out.data(), out.size(), &ol, 0);
  fprintf(stderr, "zd_decompress -> %d (%s), %zu bytes\n", st, zd_status_name(st), ol);
  if (argc > 2) { FILE* o = fopen(argv[2], "wb"); fwrite(out.data(), 1, ol, o); fclose(o); }
  return st ? 1 : 0;
}
