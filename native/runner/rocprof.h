// rocprofv3 integration of the runner: DSTACK_ROCPROF=1 wraps the job in kernel-trace statistics,
// DSTACK_ROCPROF_COUNTERS adds hardware counters (--pmc) in the same pass; the summaries are
// appended to the job log when the job ends (SURVEY §2.I "rocprof counters in run logs").
#pragma once
#include <string>
#include <vector>

namespace dsa {

// "SQ_WAVES, TCC_HIT_sum GRBM_GUI_ACTIVE" -> {"SQ_WAVES", "TCC_HIT_sum", "GRBM_GUI_ACTIVE"}
std::vector<std::string> split_counters(const std::string& spec);

// A --pmc set rocprofv3 can collect in ONE pass on CDNA3/4.  rocprofv3 does not split counters
// over passes: asked for more than a block holds it fails and can hang, so the runner checks the
// per-block budget first -- SQ 8, TCC 4 (FETCH_SIZE takes 3, WRITE_SIZE 2), TCP 4, TA 2, TD 2,
// GRBM 2; _sum/_avr/_min/_max of one counter count once.  Unknown derived metrics are rejected
// (their hardware cost is not known here).
bool validate_pmc(const std::vector<std::string>& counters, std::string& err);

// rocprofv3 argv prefix for the job ("rocprofv3 --kernel-trace --stats [--pmc ...] ... --")
std::vector<std::string> rocprof_argv(const std::string& out_dir, const std::vector<std::string>& counters);

// one CSV record (quoted fields with commas / doubled quotes, as rocprofv3 writes kernel names)
std::vector<std::string> parse_csv_record(const std::string& line);

// job-log text: the top `top` rows of *_kernel_stats.csv
std::string summarize_kernel_stats(const std::string& csv, int top);
// job-log text: per kernel, each counter summed over its dispatches (*_counter_collection.csv),
// kernels ordered by the first counter, top `top`
std::string summarize_counters(const std::string& csv, const std::vector<std::string>& counters, int top);

}  // namespace dsa
