// mrgpu -- command-line driver over libmrgpu.so, mirroring the reference's process UX:
//   mrworker <map_n> <reduce_n>   (src/bin/mrworker.rs:10-17): inputs data/gut-{m}.txt for m < map_n,
//   outputs mr-{r}.txt in the working directory (src/mr/worker.rs:67, 167).
// The coordinator's task assignment (src/mr/coordinator.rs:137-215) becomes a static plan over N GPUs
// (one host thread each): GPU g maps files m % N == g and reduces partitions r % N == g, and the
// map -> reduce hand-off is an RCCL all-to-all over xGMI (mrg_job_shuffle).
// --final also writes final.txt, the output of src/run.sh:16-20 (cat mr-* | sort, LC_ALL=C), built on the GPUs.
// --times prints the wall-clock phases of the job (mrg_run_get_stats) as one JSON line on stderr.
//   usage: mrgpu <map_n> <reduce_n> [--gpus N] [--app wc|indexer] [--no-compat-drop-last] [--final] [--times]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "mrgpu.h"

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "Usage: mrgpu <input files number> <reduce task number> [--gpus N] [--app wc|indexer] "
                        "[--no-compat-drop-last] [--final] [--times]\n");
        return 2;
    }
    const int map_n = atoi(argv[1]);
    const int reduce_n = atoi(argv[2]);
    int app = MRG_APP_WC, gpus = 1;
    uint32_t flags = 0;
    bool times = false;
    for (int i = 3; i < argc; ++i) {
        if (!strcmp(argv[i], "--app") && i + 1 < argc) {
            ++i;
            app = !strcmp(argv[i], "indexer") ? MRG_APP_INDEXER : MRG_APP_WC;
        } else if (!strcmp(argv[i], "--gpus") && i + 1 < argc) {
            gpus = atoi(argv[++i]);
        } else if (!strcmp(argv[i], "--no-compat-drop-last")) {
            flags |= MRG_FLAG_NO_COMPAT_DROP_LAST;
        } else if (!strcmp(argv[i], "--final")) {
            flags |= MRG_FLAG_FINAL_TXT;
        } else if (!strcmp(argv[i], "--times")) {
            times = true;
        } else {
            fprintf(stderr, "mrgpu: unknown argument %s\n", argv[i]);
            return 2;
        }
    }
    if (map_n < 0 || reduce_n <= 0 || gpus < 1) {
        fprintf(stderr, "bad task counts\n");
        return 2;
    }
    printf("[Worker Configuration] #%d Map Tasks | #%d Reduce Tasks | %d GPU(s)\n", map_n, reduce_n, gpus);
    std::vector<std::string> names;
    for (int m = 0; m < map_n; ++m) names.push_back("data/gut-" + std::to_string(m) + ".txt");
    std::vector<const char *> files;
    for (auto &n : names) files.push_back(n.c_str());
    const int rc = mrg_run_job(files.data(), files.size(), (uint32_t)reduce_n, app, ".", flags, gpus);
    if (rc) {
        fprintf(stderr, "mrgpu: error %d: %s\n", rc, mrg_last_error());
        return 1;
    }
    if (times) {
        mrg_run_stats st;
        if (mrg_run_get_stats(&st) == MRG_OK)
            fprintf(stderr,
                    "{\"ms_total\": %.3f, \"ms_open\": %.3f, \"ms_read\": %.3f, \"ms_map\": %.3f, \"ms_shuffle\": %.3f, "
                    "\"ms_reduce\": %.3f, \"ms_write\": %.3f, \"input_bytes\": %llu, \"output_bytes\": %llu, \"n_gpus\": %d}\n",
                    st.ms_total, st.ms_open, st.ms_read, st.ms_map, st.ms_shuffle, st.ms_reduce, st.ms_write,
                    (unsigned long long)st.input_bytes, (unsigned long long)st.output_bytes, st.n_gpus);
    }
    return 0;
}
