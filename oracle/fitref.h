/* oracle/fitref.h — CPU restatement of the reference path (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so.
 * The product (slurm-bridge-operator_amd/, libfitgpu.so) never links or calls anything here.
 *
 * Parity status:
 *   - ref_parse_duration / ref_parse_resources / ref_parse_partitions_names: PINNED by the
 *     reference's own Go tests (pkg/slurm-agent/parse_test.go:26-122, :224-258, :296-314),
 *     committed as tests/golden/reference_vectors.json.
 *   - ref_parse_node / ref_parse_partition / ref_split_records / demand derivation / capacity:
 *     restated line-by-line from the reference; the reference has no tests for them, so they are
 *     pinned only by build-authored fixtures ("parity unpinned" vs the reference itself).
 *   - ref_place (sequential priority-order best fit): the reference has NO J×N fit loop
 *     (SURVEY.md §8 a13/a14); it follows DESIGN.md §2 (SPEC).  Parity unpinned vs the reference;
 *     pinned by hand-computed vectors + an independent pure-Python restatement (tests/).
 */
#ifndef FITREF_H
#define FITREF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ParseDuration (pkg/slurm-agent/parse.go:36-109). 0 ok, 1 ErrDurationIsUnlimited, -1 error. */
int ref_parse_duration(const char* s, int64_t* out_ns);

typedef struct {
    int64_t nodes, mem_per_node, cpu_per_node, wall_ns;
} ref_resources;
/* parseResources (parse.go:111-190). 0 ok, -1 error. */
int ref_parse_resources(const char* text, ref_resources* out);

/* parsePartitionsNames (parse.go:192-210): writes NUL-separated names into buf, returns count
 * (or -1 if buf too small). */
int ref_parse_partitions_names(const char* raw, char* buf, int buflen);

/* parsePartition (parse.go:278-289): Nodes= values split on ',' (no hostlist expansion). */
int ref_parse_partition(const char* raw, char* buf, int buflen);

typedef struct {
    int64_t cpus, memory, gpus, allo_cpus, allo_memory, allo_gpus;
} ref_node;
/* parseNode (parse.go:291-308). */
void ref_parse_node(const char* raw, ref_node* out);
/* Client.Nodes record loop (slurm.go:354-363): returns number of records parsed (<= cap). */
int ref_parse_nodes(const char* scontrol_out, ref_node* out, int cap);

/* Operator demand derivation (pkg/slurm-bridge-operator/parse.go:30-135, pod.go:70-162). */
typedef struct {
    int64_t nodes, cpus_per_task, ntasks, ntasks_per_node, mem_per_cpu, wall_ns;
    char array[64];
} ref_job_resources;
/* extractBatchResourcesFromScript: 0 ok, -1 error, -3 = the reference panics (index out of range). */
int ref_extract_batch_resources(const char* script, ref_job_resources* out);
void ref_apply_spec_and_defaults(ref_job_resources* r, int64_t nodes, int64_t cpus_per_task,
                                 int64_t mem_per_cpu, int64_t ntasks_per_node, const char* array,
                                 int64_t ntasks);
int64_t ref_parse_array_len(const char* array);
/* genResourceListForPod (pod.go:143-162): cpu count and memory quantity (bytes, as the ref). */
void ref_pod_request(const ref_job_resources* r, int64_t* cpu, int64_t* memory);
/* DESIGN.md §2 per-node demand; Slurm --array task count; a pod's admission requests. */
int ref_job_demand(const ref_job_resources* r, int32_t* cpu, int32_t* mem, int32_t* wall,
                   uint16_t* k);
int ref_array_tasks(const char* array, int64_t* tasks, int64_t* running);
int ref_pod_demand(const char* const* labels, const char* script, int64_t max_array_size, int32_t* out,
                   int cap);
/* GetPartitionCapacity (pkg/slurm-virtual-kubelet/node.go:169-199). */
void ref_partition_capacity(const ref_node* nodes, int n, int64_t* cpu, int64_t* memory,
                            int64_t* gpu, int64_t* pods);

/* SPEC sequential priority-order best fit.  out[j*kmax+i]: node id, -1 unplaced,
 * -2 rejected by partition limits.  Node columns are updated in place.  Returns 0, or -1 on
 * invalid input.  stats (optional, 4 entries): placed, unplaced, rejected, evals. */
int ref_place(int32_t n, int32_t* cpu_free, int32_t* mem_free, int32_t* gpu_free,
              const int32_t* avail_min, const uint32_t* part_mask,
              int32_t p, const int32_t* max_time, const int32_t* max_cpus, const int32_t* max_mem,
              int32_t j, const int32_t* cpu, const int32_t* mem, const int32_t* gpu,
              const int32_t* wall, const uint16_t* part, const uint16_t* nodes_k, int32_t kmax,
              int32_t* out, int64_t* stats);

/* Score / key of one (job, node) pair: UINT64_MAX when infeasible. */
uint64_t ref_key(int32_t node_id, int32_t cpu_free, int32_t mem_free, int32_t gpu_free,
                 int32_t avail, uint32_t mask, int32_t cpu, int32_t mem, int32_t gpu, int32_t wall,
                 int32_t part);

/* ---- SPEC §2b time-windowed backfill (oracle/fitref_tl.c) — parity unpinned vs the reference,
 * which has no reservation timeline.  tl: dense [n][H][3] (cpu, mem, gpu). */
int ref_build_timeline(int32_t n, int32_t H, int32_t slot_min, const int32_t* cpu_free,
                       const int32_t* mem_free, const int32_t* gpu_free, const int32_t* avail_min,
                       const int32_t* rel_off, const int32_t* rel_slot, const int32_t* rel_cpu,
                       const int32_t* rel_mem, const int32_t* rel_gpu, int32_t* tl);
int32_t ref_slots(int32_t wall, int32_t slot_min);
uint64_t ref_key_tl(int32_t x, int32_t H, const int32_t* row, uint32_t mask, int32_t cpu,
                    int32_t mem, int32_t gpu, int32_t d, int32_t part, int32_t* out_start);
int ref_place_tl(int32_t n, int32_t H, int32_t slot_min, int32_t* tl, const uint32_t* part_mask,
                 int32_t p, const int32_t* max_time, const int32_t* max_cpus,
                 const int32_t* max_mem, int32_t j, const int32_t* cpu, const int32_t* mem,
                 const int32_t* gpu, const int32_t* wall, const uint16_t* part, int32_t* out_node,
                 int32_t* out_start, int64_t* stats);

/* splitmix64 twin of fitgpu/synth.py (rnd / uni). */
uint64_t ref_rnd(uint64_t seed, uint32_t stream, uint64_t idx);

#ifdef __cplusplus
}
#endif
#endif
