// TEST INFRASTRUCTURE: run the emulated checker on JSONL files.
#include <stdio.h>
#include <string.h>

#include "s2lincheck.h"

int main(int argc, char** argv) {
  s2lc_opts o;
  memset(&o, 0, sizeof o);
  o.struct_size = sizeof o;
  o.device = -1;
  int st = 0;
  s2lc_ctx* ctx = s2lc_create(&o, &st);
  if (!ctx) { fprintf(stderr, "create %d\n", st); return 2; }
  for (int i = 1; i < argc; ++i) {
    char err[512];
    s2lc_history* h = nullptr;
    int rc = s2lc_load_jsonl(argv[i], nullptr, 0, &h, err, sizeof err);
    if (rc) { fprintf(stderr, "%s: load %d %s\n", argv[i], rc, err); continue; }
    s2lc_result r;
    rc = s2lc_check(ctx, h, &r);
    printf("%s rc=%d verdict=%d reason=%d configs=%llu rounds=%u witness=%u\n", argv[i], rc, r.verdict, r.reason,
           (unsigned long long)r.configs_explored, r.rounds, r.witness_len);
    s2lc_result_free(&r);
    s2lc_history_free(h);
  }
  s2lc_destroy(ctx);
  return 0;
}
