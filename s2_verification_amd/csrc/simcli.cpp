// simcli.cpp — s2-simulate: the collector's command line
// (rust/s2-verification/src/bin/collect-history.rs:33-43) over the
// deterministic S2 simulator instead of a live S2 stream (out of scope here,
// SURVEY.md §8). Writes ./data/records.<epoch>.jsonl in the collector's
// Start/Finish schema and prints the path, as collect-history does.
//
//   s2-simulate <basin> <stream> [--num-concurrent-clients N] [--num-ops-per-client M]
//               [--workflow regular|match-seq-num|fencing] [--seed S]
//               [--p-indefinite P] [--p-definite P] [--initial-records R]
//               [--max-client-ids N] [--violation none|read-hash|definite-applied|tail|stale-msn]
//               [--output PATH]
// (basin / stream name the stream a live run would use; they are accepted and
// ignored.)
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>

#include <string>

#include "s2lincheck.h"

static int usage(const char* a0) {
  fprintf(stderr,
          "usage: %s <basin> <stream> [--num-concurrent-clients N] [--num-ops-per-client M]\n"
          "       [--workflow regular|match-seq-num|fencing] [--seed S] [--p-indefinite P] [--p-definite P]\n"
          "       [--initial-records R] [--max-client-ids N]\n"
          "       [--violation none|read-hash|definite-applied|tail|stale-msn] [--output PATH]\n",
          a0);
  return 2;
}

int main(int argc, char** argv) {
  s2lc_sim_params p;
  s2lc_sim_params_default(&p);
  p.num_clients = 5;       // collect-history.rs:38 default
  p.ops_per_client = 100;  // collect-history.rs:40 default
  p.seed = (uint64_t)time(nullptr);
  std::string out;
  int positional = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    std::string v;
    const size_t eq = a.find('=');
    if (a.rfind("--", 0) == 0 && eq != std::string::npos) {
      v = a.substr(eq + 1);
      a = a.substr(0, eq);
    } else if (a.rfind("--", 0) == 0) {
      if (a == "--help" || a == "-h") return usage(argv[0]), 0;
      if (i + 1 >= argc) return usage(argv[0]);
      v = argv[++i];
    } else {
      ++positional;
      continue;
    }
    if (a == "--num-concurrent-clients") p.num_clients = (uint32_t)strtoul(v.c_str(), nullptr, 10);
    else if (a == "--num-ops-per-client") p.ops_per_client = (uint32_t)strtoul(v.c_str(), nullptr, 10);
    else if (a == "--seed") p.seed = strtoull(v.c_str(), nullptr, 10);
    else if (a == "--p-indefinite") p.p_indefinite = strtod(v.c_str(), nullptr);
    else if (a == "--p-definite") p.p_definite = strtod(v.c_str(), nullptr);
    else if (a == "--initial-records") p.initial_records = strtoull(v.c_str(), nullptr, 10);
    else if (a == "--max-client-ids") p.max_client_ids = (uint32_t)strtoul(v.c_str(), nullptr, 10);
    else if (a == "--output") out = v;
    else if (a == "--workflow") {
      if (v == "regular") p.workflow = S2LC_WF_REGULAR;
      else if (v == "match-seq-num") p.workflow = S2LC_WF_MATCH_SEQ_NUM;
      else if (v == "fencing") p.workflow = S2LC_WF_FENCING;
      else return usage(argv[0]);
    } else if (a == "--violation") {
      if (v == "none") p.violation = S2LC_VIOL_NONE;
      else if (v == "read-hash") p.violation = S2LC_VIOL_READ_HASH;
      else if (v == "definite-applied") p.violation = S2LC_VIOL_DEFINITE_APPLIED;
      else if (v == "tail") p.violation = S2LC_VIOL_TAIL;
      else if (v == "stale-msn") p.violation = S2LC_VIOL_STALE_MSN;
      else return usage(argv[0]);
    } else {
      return usage(argv[0]);
    }
  }
  if (positional != 2 || p.num_clients == 0) return usage(argv[0]);
  uint8_t* buf = nullptr;
  size_t len = 0;
  if (s2lc_simulate_jsonl(&p, &buf, &len) != 0) {
    fprintf(stderr, "simulation failed\n");
    return 1;
  }
  if (out.empty()) {  // collect-history.rs: ./data/records.<epoch secs>.jsonl
    if (mkdir("./data", 0755) != 0 && errno != EEXIST) { perror("mkdir ./data"); return 1; }
    out = "./data/records." + std::to_string((long long)time(nullptr)) + ".jsonl";
  }
  FILE* f = fopen(out.c_str(), "ab");
  if (!f || fwrite(buf, 1, len, f) != len || fclose(f) != 0) {
    perror(out.c_str());
    s2lc_free(buf);
    return 1;
  }
  s2lc_free(buf);
  printf("%s\n", out.c_str());
  return 0;
}
