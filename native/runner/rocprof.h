// rocprofv3 integration of the runner: DSTACK_ROCPROF=1 wraps the job in kernel-trace statistics,
// DSTACK_ROCPROF_COUNTERS adds hardware counters (--pmc) in the same pass; the summaries are
// appended to the job log when the job ends (SURVEY §2.I "rocprof counters in run logs").
#pragma once
#include <functional>
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

// rocprofv3 argv prefix for the job ("rocprofv3 --kernel-trace --stats [--pmc ...] ... --"); every
// profiled process writes <out_dir>/job_<pid>_{kernel_stats,counter_collection}.csv
std::vector<std::string> rocprof_argv(const std::string& out_dir, const std::vector<std::string>& counters);

// Put rocprofv3 directly in front of the job's GPU program.  rocprofv3's preloaded library
// initialises the GPU in the process it is given (with --pmc it always does), so whatever follows
// "--" must be the GPU program itself: a shell, `env`, `timeout` or a launcher there would fork or
// exec a GPU program from a process that has already touched the GPU.  `rp` is rocprof_argv()'s
// prefix (ending in "--").
//  * job = {shell, "-c", script} (how the server runs `commands`): the script's LAST simple command
//    becomes `[VAR=x ...] exec rocprofv3 ... -- prog args`, so the shell (which never touches the GPU)
//    execs rocprofv3, which execs the program;
//  * that command is `torchrun ... script.py` / `python -m torch.distributed.run ...`: each rank
//    is profiled instead -- `torchrun ... --no-python rocprofv3 ... -- python3 -u script.py`, the
//    launcher itself stays outside the profiler;
//  * job = {prog, args...} (an entrypoint without a shell): rocprofv3 ... -- prog args.
// Anything else -- a last command that is a wrapper (bash, sh, env, timeout, numactl, mpirun, ...),
// a pipeline, a background job, a compound command, one reached through `||` -- is refused with a
// reason, and the caller runs the job unprofiled.
//
// The program after "--" is also checked on disk (`look`): it must be an ELF binary, or a "#!"
// script whose interpreter is Python (rewritten to `<interpreter> script args`, so the Python
// binary -- checked to be ELF too -- is what rocprofv3 starts); a shell script, an `env bash`
// shebang, a pyenv-style shim or a program that cannot be found is refused.  `accelerate launch`
// and `deepspeed` are profiled per rank like torchrun (`--no_python rocprofv3 ... -- <python> -u
// script.py`); uv/poetry/conda/pixi/pipenv/hatch runners and `python -m <launcher>` are refused.
// A script with a heredoc (`<<`) is refused (its body lines are not commands).
struct ProgramInfo {
  bool found = false;
  std::string path;  // resolved file
  std::string head;  // its first bytes (up to 256)
};
// resolve a program word (a path, or a name looked up on PATH) against `cwd`
using ProgramLookup = std::function<ProgramInfo(const std::string& prog, const std::string& cwd)>;
// the runner's lookup: `path_env` (the job's PATH) and the real filesystem
ProgramLookup fs_program_lookup(const std::string& path_env);

bool rocprof_wrap(const std::vector<std::string>& job, const std::vector<std::string>& rp,
                  std::vector<std::string>& out, std::string& err, const ProgramLookup& look,
                  const std::string& cwd);

// one CSV record (quoted fields with commas / doubled quotes, as rocprofv3 writes kernel names)
std::vector<std::string> parse_csv_record(const std::string& line);

// job-log text: per kernel, calls and time summed over every *_kernel_stats.csv (one per profiled
// process: torchrun ranks each write their own), top `top` by total time
std::string summarize_kernel_stats(const std::vector<std::string>& csvs, int top);
// job-log text: per kernel, each counter summed over its dispatches in every
// *_counter_collection.csv, kernels ordered by the first counter, top `top`
std::string summarize_counters(const std::vector<std::string>& csvs, const std::vector<std::string>& counters,
                               int top);

}  // namespace dsa
