/* fitgpu.h — C-ABI of the MI355X batched job→node placement engine (libfitgpu.so).
 *
 * This is the cgo seam of the new pkg/fitgpu.  The reference has no fit loop
 * of its own (capacity is summed in pkg/slurm-virtual-kubelet/node.go:169-199 and the fit runs in
 * the external kube-scheduler), so the placement entry points replace *that decision*; the
 * ingest / demand / capacity entry points replace the Go functions cited on each declaration.
 * The slurm-agent gRPC API (pkg/workload/workload.proto:23-62) and the virtual-kubelet provider
 * interface (pkg/slurm-virtual-kubelet/provider.go:26) are unchanged; INTEGRATION.md shows the
 * cgo binding and the call sites.
 *
 * Conventions
 *   - Plain pointers and sizes only.  The caller owns every buffer; the library copies inputs in
 *     during the call and never retains a caller pointer (cgo rule).
 *   - Return 0 on success, a negative FIT_E_* code on failure; fit_strerror() gives the text and
 *     fit_last_error() the detail of the last failure on the calling thread.  No C++ exception
 *     crosses the ABI.  There is no CPU fallback: without a usable gfx950 device fit_create fails.
 *   - A fit_ctx must not be used by two threads at once; several contexts may coexist.
 *   - Units: cpus, MiB, GPUs (gres/gpu count), minutes.  INT32_MAX avail = none.
 */
#ifndef FITGPU_H
#define FITGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FITGPU_ABI_VERSION 8

/* ---- error codes ---------------------------------------------------------------------- */
#define FIT_OK 0
#define FIT_E_INVAL (-1)       /* invalid argument or input value                          */
#define FIT_E_HIP (-2)         /* HIP runtime error                                        */
#define FIT_E_RCCL (-3)        /* RCCL (collective) error                                  */
#define FIT_E_OOM (-4)         /* device or host allocation failed                         */
#define FIT_E_NODEV (-5)       /* no usable gfx950 device                                  */
#define FIT_E_STATE (-6)       /* call out of order (e.g. fit_place before fit_load_nodes) */
#define FIT_E_PARSE (-7)       /* malformed text (ingest helpers)                          */
#define FIT_E_UNLIMITED (-8)   /* ParseDuration: ErrDurationIsUnlimited                    */

/* ---- placement result codes (out_node entries) ------------------------------------------ */
#define FIT_UNPLACED (-1)  /* no node (or not enough distinct nodes) fits at this point     */
#define FIT_REJECTED (-2)  /* violates the partition's MaxTime/MaxCPUsPerNode/MaxMemPerNode  */

#define FIT_MAX_PARTITIONS 32
#define FIT_MAX_K 8         /* nodes per job (--nodes) supported by fit_place              */
#define FIT_MAX_NODES (1 << 29) /* node rows per fit_load_nodes (commit keys tag pos << 3)  */

typedef struct fit_ctx fit_ctx;

/* Optional host-side exchange used instead of RCCL (world > 1): tests run several ranks on one
 * GPU with it, a caller may route the exchange through its own transport.  In-place on host
 * memory; return 0 on success.  ops: */
#define FIT_XCHG_ALLGATHER_U64 1  /* buf holds world*count u64, this rank's block at rank*count */
#define FIT_XCHG_MIN_U64 2        /* elementwise min over ranks, count u64                    */
#define FIT_XCHG_MAX_I32 3        /* elementwise max over ranks, count int32                  */
#define FIT_XCHG_MIN_I32 4        /* elementwise min over ranks, count int32                  */
typedef int (*fit_exchange_fn)(void* user, int op, void* buf, int64_t count);

typedef struct {
    int32_t device;       /* HIP device ordinal; -1 = current device                        */
    int32_t rank;         /* this process' rank in a node-sharded group (0 if world == 1)  */
    int32_t world;        /* number of GPUs sharing one placement (1 = single GPU)         */
    const void* nccl_id;  /* 128-byte ncclUniqueId from fit_nccl_unique_id() when world>1 */
    int32_t shard_mode;   /* FIT_SHARD_*: how world > 1 ranks split one placement           */
    int32_t window_min;   /* jobs per component per round, lower bound (0 = default 256)   */
    int32_t window_max;   /* upper bound (0 = default 8192)                                 */
    int32_t flags;        /* FIT_FLAG_* bits, 0 = none                                      */
    fit_exchange_fn exchange;  /* NULL = RCCL over xGMI (nccl_id required)                  */
    void* exchange_user;
} fit_opts;

/* fit_opts.flags: run the multi-rank code path (shard split, per-round exchange, merge) even at
 * world == 1, over a one-rank RCCL communicator (or the host exchange): exercises the collective
 * calls on a single GPU.  Placements are identical to the default path. */
#define FIT_FLAG_COLLECTIVES 1

#define FIT_SHARD_AUTO 0       /* components if there are at least `world` of them, else nodes */
#define FIT_SHARD_NODES 1      /* every rank scans 1/world of every component's nodes; per     */
                               /* round: allgather candidates + 64-bit min-allreduce of bounds */
#define FIT_SHARD_COMPONENTS 2 /* ranks own whole partition components; one merge at the end   */

typedef struct {
    int64_t jobs;          /* jobs in the call                                              */
    int64_t placed;        /* jobs placed                                                    */
    int64_t unplaced;      /* FIT_UNPLACED                                                   */
    int64_t rejected;      /* FIT_REJECTED                                                   */
    int64_t rounds;        /* speculative rounds executed                                    */
    int64_t evals;         /* (job, node) fit evaluations performed by this rank's scans     */
    int64_t useful_evals;  /* J_active × N: the single-pass work of the naive scalar path    */
    int64_t stops_rescan;  /* round cut because a job's candidate list ran out               */
    int64_t stops_dirty;   /* round cut because the dirty-node set was full                  */
    double ms_total;       /* wall time of the call on the host clock                        */
    double ms_scan;        /* scan time: k_scan launches (host loop) or the average scan-   */
                           /* worker busy time inside the persistent engine                 */
    double ms_commit;      /* commit time: k_commit launches, or the slowest component's     */
                           /* committer inside the persistent engine                        */
    double ms_exchange;    /* device time in the RCCL exchange (world > 1)                   */
    double ms_device;      /* device time of the placement launches (HIP events)             */
    int32_t shard_mode;    /* mode used (FIT_SHARD_NODES / FIT_SHARD_COMPONENTS; 0 if world 1) */
    int32_t components;    /* independent partition components                               */
    int32_t engine;        /* 1: persistent single-launch engine (k_engine); 0: host-driven rounds; */
                           /* 2: direct small placement (k_small, <= FIT_SMALL_DIRECT jobs);         */
                           /* 3: demand-class engine (k_class: by default when the live jobs are at  */
                           /*    least half multi-node; FIT_CLASS=1 / 0 forces it on / off)          */
    int32_t reserved;
    double ms_arb_wait;    /* host time waiting for the device's persistent-launch lock: one   */
                           /* persistent launch per GPU at a time, across contexts and processes */
} fit_stats;

/* ---- engine -------------------------------------------------------------------------- */
int fit_create(const fit_opts* opts, fit_ctx** out_ctx);
void fit_destroy(fit_ctx* ctx);
int fit_abi_version(void);
const char* fit_strerror(int code);
const char* fit_last_error(void);
/* 128-byte RCCL unique id for a node-sharded group (rank 0 creates, everyone passes it). */
int fit_nccl_unique_id(void* out128);
/* Watchdog of the persistent engines: every device-side wait gives up after `us` microseconds
 * (default 10 s, or FIT_WATCHDOG_MS); us <= 0 restores the default.  A trip fails the call with
 * FIT_E_HIP, fit_last_error() names the wait (site, component, round, tile, ring indices, how long
 * it waited), and the context stays usable: fit_place restores the node table it started from;
 * fit_place_tl drops the timeline (FIT_E_STATE until fit_load_timeline).  Persistent launches of
 * all contexts on one GPU — in every process — run one at a time (a per-device lock file in
 * fit_lock_dir(); fit_stats.ms_arb_wait). */
int fit_set_watchdog_us(fit_ctx* ctx, int64_t us);
/* The directory of the per-GPU lock file that serialises persistent launches across processes:
 * FIT_LOCK_DIR if set; else /var/run/fitgpu when it is a directory (the hostPath volume every
 * virtual-kubelet pod of a host mounts: INTEGRATION.md item 6); else /tmp.  Writes it (NUL-
 * terminated) into buf and returns 0 when the directory is the configured or default shared one,
 * 1 when it fell back to /tmp — private to one pod in the reference's deployment (one VK pod per
 * partition, pkg/configurator/configurator.go:188-293), so VKs in other pods on the same GPU are
 * NOT arbitrated: the caller should warn.  FIT_E_INVAL: buf too small.  No device needed. */
int fit_lock_dir(char* buf, int32_t buflen);

/* Node table: one row per Slurm node, in Client.Nodes output order (pkg/slurm-agent/slurm.go:
 * 343-364); the row index is the node id placements refer to.  free = total - alloc (the
 * Node{Cpus,AlloCpus,Memory,AlloMemory,Gpus,AlloGpus} of workload.proto:165-174).  part_mask bit
 * p = member of partition p.  Host pointers. */
int fit_load_nodes(fit_ctx* ctx, int32_t n, const int32_t* cpu_free, const int32_t* mem_free,
                   const int32_t* gpu_free, const int32_t* avail_min, const uint32_t* part_mask);
/* Same, but the columns are device pointers (already resident in HBM on this context's GPU). */
int fit_load_nodes_device(fit_ctx* ctx, int32_t n, const int32_t* cpu_free,
                          const int32_t* mem_free, const int32_t* gpu_free,
                          const int32_t* avail_min, const uint32_t* part_mask);

/* Partition limits from parseResources (pkg/slurm-agent/parse.go:111-190) after the agent's
 * override merge (pkg/slurm-agent/api/slurm.go:297-341): -1 = UNLIMITED.  Minutes / CPUs / MiB. */
int fit_load_partitions(fit_ctx* ctx, int32_t p, const int32_t* max_time_min,
                        const int32_t* max_cpus_per_node, const int32_t* max_mem_per_node);

/* Place J jobs in priority order (index order) with sequential best-fit semantics.
 * Demands are per node; nodes_k (may be NULL = all 1) is the --nodes count, 0 treated as 1.
 * out_node[j*kmax + i], i < nodes_k[j]: node id, FIT_UNPLACED or FIT_REJECTED; other entries -1.
 * The context's node table is updated (jobs consume resources).  Host pointers. */
int fit_place(fit_ctx* ctx, int32_t j, const int32_t* cpu, const int32_t* mem, const int32_t* gpu,
              const int32_t* wall, const uint16_t* part, const uint16_t* nodes_k, int32_t kmax,
              int32_t* out_node, fit_stats* stats);
/* Same with device pointers (inputs resident in HBM, output written in HBM). */
int fit_place_device(fit_ctx* ctx, int32_t j, const int32_t* cpu, const int32_t* mem,
                     const int32_t* gpu, const int32_t* wall, const uint16_t* part,
                     const uint16_t* nodes_k, int32_t kmax, int32_t* out_node, fit_stats* stats);

/* Current (post-placement) free columns, in node-id order.  Host pointers, n entries each. */
int fit_read_nodes(fit_ctx* ctx, int32_t* cpu_free, int32_t* mem_free, int32_t* gpu_free);
/* Free capacity per partition (Σ over member nodes of the current free columns): the engine's
 * replacement for the allocation-blind sum of GetPartitionCapacity (node.go:183-190). */
int fit_partition_free(fit_ctx* ctx, int32_t p, int64_t* cpu, int64_t* mem_mib, int64_t* gpu);

/* ---- time-windowed backfill (BASELINE config C5) -------------------------
 * Each node's free resources over a horizon of `slots` slots of `slot_min` minutes (slots <=
 * 1024): the node table of the last fit_load_nodes is the state at slot 0, and the jobs already
 * running hand resources back at their end — release events, CSR by node id: node x's events are
 * [rel_off[x], rel_off[x+1]) with non-decreasing rel_slot (slot <= 0 = already free) and amounts
 * >= 0.  A node is usable for slots t < avail_min / slot_min.  Call after fit_load_nodes (which
 * drops the timeline); rel_off NULL = no releases.  Host pointers; rel_off has n+1 entries.
 * The walltime source is the job's --time (pkg/slurm-bridge-operator/parse.go:84-91) and the
 * squeue EndTime of running jobs; the partition MaxTime check is parseResources' (parse.go:128-138). */
int fit_load_timeline(fit_ctx* ctx, int32_t slots, int32_t slot_min, const int32_t* rel_off,
                      const int32_t* rel_slot, const int32_t* rel_cpu, const int32_t* rel_mem,
                      const int32_t* rel_gpu);
/* Same with device pointers; n_rel = rel_off[n] (the caller knows it; not read back). */
int fit_load_timeline_device(fit_ctx* ctx, int32_t slots, int32_t slot_min,
                             const int32_t* rel_off, int64_t n_rel, const int32_t* rel_slot,
                             const int32_t* rel_cpu, const int32_t* rel_mem,
                             const int32_t* rel_gpu);
/* Sequential priority-order backfill: each job (one node, nodes_k = 1) gets the node and the
 * earliest start slot at which its demand fits for ceil(wall / slot_min) consecutive slots, best
 * fit among the nodes with that start; the reservation is committed and later
 * jobs see it.  out_node[j]: node id, FIT_UNPLACED (no start inside the horizon) or FIT_REJECTED;
 * out_start[j]: start slot, -1 when not placed.  Host pointers. */
int fit_place_tl(fit_ctx* ctx, int32_t j, const int32_t* cpu, const int32_t* mem,
                 const int32_t* gpu, const int32_t* wall, const uint16_t* part, int32_t* out_node,
                 int32_t* out_start, fit_stats* stats);
/* Same with device pointers (inputs resident in HBM, outputs written in HBM). */
int fit_place_tl_device(fit_ctx* ctx, int32_t j, const int32_t* cpu, const int32_t* mem,
                        const int32_t* gpu, const int32_t* wall, const uint16_t* part,
                        int32_t* out_node, int32_t* out_start, fit_stats* stats);
/* Release events for fit_load_timeline from the running jobs a caller knows — the virtual
 * kubelet's own pods: JobInfo.end_time and JobInfo.node_list (workload.proto:252-292; the
 * node_list expanded with fit_expand_hostlist and mapped to engine rows through the
 * fit_node_names table) and each pod's per-node demand (fit_pod_demand).  Job i holds (cpu[i],
 * mem[i], gpu[i]) on every node job_nodes[job_off[i] .. job_off[i+1]) for rem_min[i] more minutes
 * (end_time − now) and hands it back at slot max(1, ceil(rem_min / slot_min)), capped at `slots`
 * (a job past its end time holds its nodes until Slurm ends it; a release at the horizon changes
 * nothing).  Output: the CSR by node fit_load_timeline reads (rel_off[n + 1]; rel_slot / rel_cpu /
 * rel_mem / rel_gpu, slots non-decreasing per node, jobs in order within a slot), at most cap
 * events.  Returns the event count or FIT_E_INVAL (node id out of range, negative demand,
 * job_off not starting at 0 or decreasing, slots / slot_min < 1, cap too small). */
int fit_release_events(int32_t n, int32_t m, const int32_t* job_off, const int32_t* job_nodes,
                       const int64_t* rem_min, const int32_t* cpu, const int32_t* mem,
                       const int32_t* gpu, int32_t slots, int32_t slot_min, int32_t* rel_off,
                       int32_t* rel_slot, int32_t* rel_cpu, int32_t* rel_mem, int32_t* rel_gpu,
                       int32_t cap);
/* Current timelines, dense [n][slots] per column, host pointers (n * slots entries each).  Slots
 * where a node is unusable, and nodes outside every partition, read -1. */
int fit_read_timeline(fit_ctx* ctx, int32_t* cpu, int32_t* mem, int32_t* gpu);

/* ---- ingest / demand helpers (host code, mirrors of the reference Go functions) -------- */
/* ParseDuration (pkg/slurm-agent/parse.go:36-109): 0 ok, FIT_E_UNLIMITED, FIT_E_PARSE. */
int fit_parse_duration(const char* s, int64_t* out_ns);

typedef struct {
    int64_t nodes, mem_per_node, cpu_per_node, wall_ns;
} fit_resources;
/* parseResources (parse.go:111-190). */
int fit_parse_resources(const char* text, fit_resources* out);

typedef struct {
    int64_t cpus, memory, gpus, allo_cpus, allo_memory, allo_gpus;
} fit_node;
/* Client.Nodes + parseNode (slurm.go:354-363, parse.go:291-308): parses `scontrol show nodes`
 * text into at most cap records; returns the record count or a negative code. */
int fit_parse_nodes(const char* text, fit_node* out, int32_t cap);
/* parsePartition (parse.go:278-289): NUL-separated node names into buf; returns count. */
int fit_parse_partition(const char* text, char* buf, int32_t buflen);
/* parsePartitionsNames (parse.go:192-210): NUL-separated names into buf; returns count. */
int fit_parse_partitions_names(const char* text, char* buf, int32_t buflen);

typedef struct {
    int64_t nodes, cpus_per_task, ntasks, ntasks_per_node, mem_per_cpu, wall_ns;
    char array[64];
} fit_job_resources;
/* extractBatchResourcesFromScript (pkg/slurm-bridge-operator/parse.go:30-69): FIT_E_PARSE where
 * the reference returns an error or panics (bare flag as the last #SBATCH token). */
int fit_extract_batch_resources(const char* script, fit_job_resources* out);
/* setRequireResourceBySpec + setDefaultRequireResource (pod.go:70-107). */
void fit_apply_spec(fit_job_resources* r, int64_t nodes, int64_t cpus_per_task,
                    int64_t mem_per_cpu, int64_t ntasks_per_node, const char* array,
                    int64_t ntasks);
/* parseArrayLen (parse.go:126-135). */
int64_t fit_array_len(const char* array);
/* genResourceListForPod (pod.go:143-162): the pod's cpu request and memory quantity (bytes). */
void fit_pod_request(const fit_job_resources* r, int64_t* cpu, int64_t* memory);
/* Engine demand vector for one (array task of a) job: DESIGN.md §2 "demand". */
int fit_job_demand(const fit_job_resources* r, int32_t* cpu, int32_t* mem_mib, int32_t* wall_min,
                   uint16_t* nodes_k);
/* GetPartitionCapacity (pkg/slurm-virtual-kubelet/node.go:169-199), reference arithmetic. */
void fit_partition_capacity(const fit_node* nodes, int32_t n, int64_t* cpu, int64_t* memory,
                            int64_t* gpu, int64_t* pods);

/* ---- node-table ingest -------------------------------------------------
 * `scontrol show nodes` text → the engine's node columns (fit_load_nodes order and meaning).
 * Records are split and CPUTot/CPUAlloc/RealMemory/AllocMem parsed exactly as Client.Nodes +
 * parseNode (slurm.go:354-363, parse.go:291-308); added: Gres/GresUsed gpu counts (gpu_free =
 * Gres − GresUsed; the reference never sets Gpus/AlloGpus), Partitions= → part_mask bit p for
 * the p-th name of `partitions` (np NUL-separated names), State (DOWN, DRAIN, FAIL, MAINT, '*'
 * not responding, ...) → part_mask 0 (never placed), NodeName → `names` (NUL-separated, may be
 * NULL).  avail_min = INT32_MAX.  Returns the record count, FIT_E_INVAL (cap / buffer too small),
 * FIT_E_PARSE (malformed gres count). */
int fit_ingest_nodes(const char* text, const char* partitions, int32_t np, int32_t cap,
                     int32_t* cpu_free, int32_t* mem_free, int32_t* gpu_free, int32_t* avail_min,
                     uint32_t* part_mask, char* names, int32_t names_len);
/* Slurm hostlist expansion ("node[01-03,7],gpu[1-2]-ib" → node01 node02 node03 node07 gpu1-ib
 * gpu2-ib), NUL-separated into buf; returns the count, FIT_E_PARSE or FIT_E_INVAL (buf too
 * small).  The fix for parsePartition's split of "Nodes=node[1-3,5]" (parse.go:278-289). */
int fit_expand_hostlist(const char* expr, char* buf, int32_t buflen);
/* The Partition RPC's node list (PartitionResponse.nodes, workload.proto; n NUL-separated entries
 * as parsePartition split them on every comma, parse.go:278-289: "node[1-3" "5]" for
 * "Nodes=node[1-3,5]") → the expanded node names, NUL-separated into buf, in hostlist order.
 * These are the names to send to the Nodes RPC (Client.Nodes, slurm.go:343-364, which joins them
 * with commas for `scontrol show nodes`); record i of its answer is name i, and a caller must
 * refuse the answer when the record count differs.  Returns the count, FIT_E_PARSE (malformed
 * hostlist, or a name listed twice), FIT_E_INVAL (buf too small: retry with a larger one). */
int fit_node_names(const char* entries, int32_t n, char* buf, int32_t buflen);

/* ---- batched admission (CreatePod's call site) -----------------
 * The virtual kubelet calls CreatePod(ctx, *v1.Pod) (pkg/slurm-virtual-kubelet/provider.go:35-60)
 * from 10 concurrent PodSyncWorkers (options/options.go:107), one pod per call; a non-nil error
 * makes the library retry the pod later.  A fit_admitter coalesces those calls: fit_admit blocks
 * while its request joins the open batch; the batch closes max_wait_us after its first request
 * (or at max_batch requests), is ordered by (priority, arrival), placed with ONE fit_place, and
 * every caller returns with its own result.  Placements consume the context's node table, so
 * later batches see them until the next fit_admitter_load_nodes (the node ticker,
 * provider.go:470-488).  All calls are thread-safe; while an admitter owns a context, use the
 * context only through it.  fit_admitter_destroy fails still-queued requests with FIT_E_STATE. */
typedef struct fit_admitter fit_admitter;
typedef struct {
    int64_t priority;  /* smaller first (e.g. pod creation time); ties keep arrival order   */
    int32_t cpu;       /* per-node demand as fit_job_demand derives it                      */
    int32_t mem_mib;
    int32_t gpu;
    int32_t wall_min;
    uint16_t part;     /* partition index (fit_load_partitions order)                       */
    uint16_t nodes_k;  /* --nodes, 0 = 1, <= FIT_MAX_K                                      */
    uint16_t flags;    /* FIT_REQ_*: set by fit_pod_demand                                   */
    uint16_t reserved;
} fit_admit_req;
/* fit_admit_req.flags: one task of an array job (an --array label or #SBATCH --array): its pod's
 * one sbatch serves every task, so fit_admitter_script never pins it to the task's nodes */
#define FIT_REQ_ARRAY 1
typedef struct {
    int32_t node[FIT_MAX_K]; /* node ids (nodes_k of them, rest -1), or node[0] = FIT_UNPLACED
                                (no capacity now: retry) / FIT_REJECTED (partition limits)  */
    int64_t batch;           /* batch sequence number (0, 1, ...)                           */
    int32_t batch_jobs;      /* requests placed together in that batch                      */
    int32_t order;           /* this request's index in the batch's placement order        */
    int64_t ticket;          /* reservation id (> 0) when placed, else 0: see "reservations" */
} fit_admit_res;
int fit_admitter_create(fit_ctx* ctx, int32_t max_batch, int32_t max_wait_us, fit_admitter** out);
/* Blocks until the request's batch is placed.  FIT_OK (result in *res), FIT_E_INVAL (bad
 * request: negative demand, nodes_k > FIT_MAX_K; not queued), FIT_E_STATE (admitter shutting
 * down / no node table), or the batch's fit_place error. */
int fit_admit(fit_admitter* a, const fit_admit_req* req, fit_admit_res* res);
/* All-or-nothing admission of n requests (the tasks of one array job, fit_pod_demand): they join
 * ONE batch, consecutively in arrival order at their own priority.  If any of them is not placed,
 * none is: every res[i].node[0] is FIT_REJECTED (some task violates the partition limits) or
 * FIT_UNPLACED, ticket 0, and the group takes nothing: the batch is placed again without it, so
 * every later request of the batch sees the table the group left untouched — the sequential
 * semantics of placing the requests one after the other (tests/test_callsite_gpu.py
 * test_groups_in_one_batch_match_oracle).  Errors as fit_admit. */
int fit_admit_group(fit_admitter* a, const fit_admit_req* reqs, int32_t n, fit_admit_res* res);
/* Replaces the node table between batches (the node ticker, provider.go:470-488).  Every open
 * reservation (admitted, neither confirmed nor released) is taken from the new table again
 * before it is loaded — Slurm does not count a job it has not allocated yet, so a refresh would
 * otherwise hand its capacity out twice. */
int fit_admitter_load_nodes(fit_admitter* a, int32_t n, const int32_t* cpu_free,
                            const int32_t* mem_free, const int32_t* gpu_free,
                            const int32_t* avail_min, const uint32_t* part_mask);
/* The same with the table's node names and provenance.  names (n NUL-separated, fit_node_names or
 * fit_ingest_nodes order; NULL = none): open reservations are carried over to the new table by
 * NAME, so a node added to or removed from the partition does not move them to another node, and
 * fit_admitter_script can pin a pod to its nodes.  flags FIT_TABLE_STATE: part_mask carries the
 * nodes' State (fit_ingest_nodes: a DOWN / DRAIN / powered-down node is in no partition), so the
 * engine never chooses a node slurmctld would refuse, and placements are pinned.  The gRPC Nodes
 * RPC's Node has no state (workload.proto:165-174): a table built from it marks a drained node
 * with free capacity schedulable, so by default its placements only gate capacity (the script is
 * not pinned); FIT_TABLE_PIN pins them anyway (the operator's choice: a pod pinned to a drained
 * node then pends in Slurm while its reservation holds the capacity, until a TTL or release).
 * generation: fit_admitter_generation() taken BEFORE the table was fetched (0 = now): a confirmed
 * reservation is dropped only by a table fetched after its confirmation (earlier tables do not
 * count the job yet), and a table older than the last one loaded is refused (FIT_E_STATE). */
#define FIT_TABLE_STATE 1
#define FIT_TABLE_PIN 2
typedef struct {
    int32_t n;
    const int32_t* cpu_free;
    const int32_t* mem_free;
    const int32_t* gpu_free;
    const int32_t* avail_min;
    const uint32_t* part_mask;
    const char* names;
    int32_t flags;
    int64_t generation;
} fit_node_table;
int fit_admitter_load_table(fit_admitter* a, const fit_node_table* t);
/* A new table generation (> every earlier one): take it before fetching a table from Slurm. */
int64_t fit_admitter_generation(fit_admitter* a);
/* The script to submit for one pod whose admission returned `tickets` (n of them): with
 * `#SBATCH --nodelist=<names>` (fit_script_with_nodelist) when the pod is one request (n == 1; an
 * array job's tasks share one sbatch and stay unpinned) and the ticket's nodes come from a named
 * table loaded with FIT_TABLE_STATE or FIT_TABLE_PIN; the script unchanged otherwise.  *pinned (may be NULL) = 1 when
 * the directive was added.  The names are those of the table the reservation lives in now, read
 * under the same lock as placements and reloads.  Returns the length written, FIT_E_INVAL (unknown
 * ticket, out too small: strlen(script) + 32 + Σ (strlen(name) + 1) suffices). */
int fit_admitter_script(fit_admitter* a, const int64_t* tickets, int32_t n, const char* script,
                        char* out, int32_t outlen, int32_t* pinned);
int fit_admitter_partition_free(fit_admitter* a, int32_t p, int64_t* cpu, int64_t* mem_mib,
                                int64_t* gpu);
/* Reservations.  A placed request holds its demand on its nodes from admission until:
 *   confirm — Slurm now counts the job (it is allocated: the agent's Nodes RPC includes it, e.g.
 *             the pod's job is RUNNING): the reservation is dropped at the next load, not
 *             re-applied (the table then carries the allocation);
 *   release — the job will not run (pod deleted, SubmitJob failed): its demand goes back to the
 *             current table before the next batch (requires a table loaded through
 *             fit_admitter_load_nodes, else FIT_E_STATE); a confirmed one is only forgotten;
 *   ttl     — fit_admitter_set_ttl(a, L), L > 0: an open reservation that L loads have
 *             re-applied is dropped (a lost confirmation cannot hold capacity forever; 0 = never).
 * FIT_E_INVAL: unknown ticket. */
int fit_admitter_confirm(fit_admitter* a, int64_t ticket);
int fit_admitter_release(fit_admitter* a, int64_t ticket);
int fit_admitter_set_ttl(fit_admitter* a, int32_t loads);
/* Open reservations / requests queued for the next batch (monitoring, tests). */
int fit_admitter_reservations(fit_admitter* a);
int fit_admitter_pending(fit_admitter* a);
void fit_admitter_destroy(fit_admitter* a);

/* ---- CreatePod call site -------------------------------------
 * What the virtual kubelet's CreatePod has in hand — the pod's sbo.kubecluster.org/<key> labels
 * (newSubmitRequestForPod, pkg/slurm-virtual-kubelet/provider.go:62-125; keys
 * pkg/common/labels.go:9-14) and its sbatch script (Containers[0].Command[0], provider.go:71) —
 * turned into engine requests, and the engine's decision written back into the script. */
typedef struct {
    const char* nodes;            /* sbo.kubecluster.org/nodes            (NULL = label absent) */
    const char* cpus_per_task;    /* sbo.kubecluster.org/cpus-per-task                          */
    const char* mem_per_cpu;      /* sbo.kubecluster.org/mem-per-cpu                            */
    const char* ntasks_per_node;  /* sbo.kubecluster.org/ntasks-per-node                        */
    const char* array;            /* sbo.kubecluster.org/array                                  */
    const char* ntasks;           /* sbo.kubecluster.org/ntask                                  */
} fit_pod_labels;
/* Slurm --array expression ("0-15", "1,3,5-7", "0-15:4", "1-100%10") → the number of distinct
 * task ids and how many may run at once (min(tasks, %limit)).  The fix of parseArrayLen
 * (pkg/slurm-bridge-operator/parse.go:126-135), which gives 0 for "1-10%2" and "1-3,5".
 * FIT_E_PARSE: malformed, or a task id above 4,194,303. */
int fit_array_tasks(const char* array, int64_t* tasks, int64_t* max_running);
/* Slurm's MaxArraySize (slurm.conf, default 1001: task ids 0 .. 1000), which fit_pod_demand
 * enforces as sbatch does.  1 <= n <= 4,194,304; returns the previous value or FIT_E_INVAL.
 * Process-wide. */
int32_t fit_set_max_array_size(int32_t n);
/* The pod's demand as sbatch sees it: the script's #SBATCH header (extractBatchResourcesFromScript,
 * parse.go:30-69: --time, --nodes, --mem-per-cpu, --cpus-per-task, --ntasks-per-node), overridden
 * by the labels (they reach sbatch as command-line flags, pkg/slurm-agent/slurm.go:189-229; a
 * value strconv.ParseInt rejects is skipped, as provider.go:74-123 logs and skips it), then the
 * operator's defaults (pod.go:97-107) and fit_job_demand's per-node rule.  An array job becomes
 * one request per task that may run at once (fit_array_tasks; each task runs on its own nodes).
 * Writes min(n, cap) requests (partition `part`, priority `priority`) and returns n >= 1, or
 * FIT_E_PARSE (malformed #SBATCH header or array) / FIT_E_INVAL (demand out of range, or an array
 * task id >= MaxArraySize: sbatch would refuse the job, fit_set_max_array_size). */
int fit_pod_demand(const fit_pod_labels* labels, const char* script, uint16_t part,
                   int64_t priority, fit_admit_req* out, int32_t cap);
/* The script with `#SBATCH --nodelist=<names of node[0..k)>` added as the last line of its
 * #SBATCH header (after the last header line, so it overrides an earlier --nodelist / -w and the
 * header stays contiguous for extractBatchResourcesFromScript), so slurmctld allocates the nodes
 * the engine reserved — SubmitJobRequest.script (workload.proto:66), no proto change.  names: the
 * node table's names, NUL-separated in node-id order (fit_ingest_nodes, or the Partition RPC's
 * list), n_names of them.  Returns the length written (NUL-terminated), FIT_E_INVAL (a node id
 * out of range, or out too small: it needs strlen(script) + 32 + Σ (strlen(name) + 1)). */
int fit_script_with_nodelist(const char* script, const char* names, int32_t n_names,
                             const int32_t* node, int32_t k, char* out, int32_t outlen);
/* ResourcesResponse (workload.proto:137-148, filled by pkg/slurm-agent/api/slurm.go:297-341:
 * wallTime in seconds, 0 when UNLIMITED; cpuPerNode / memPerNode, -1 or 0 when unlimited or
 * unset) → fit_load_partitions' limits (minutes rounded up, -1 = no limit). */
int fit_partition_limits(int64_t wall_time_s, int64_t cpu_per_node, int64_t mem_per_node,
                         int32_t* max_time_min, int32_t* max_cpus_per_node,
                         int32_t* max_mem_per_node);
/* NodesResponse rows (workload.proto:165-174, as fit_node) → fit_load_nodes columns: free =
 * total − alloc clamped to int32, avail_min = INT32_MAX, part_mask for every row. */
int fit_node_columns(const fit_node* nodes, int32_t n, uint32_t part_mask, int32_t* cpu_free,
                     int32_t* mem_free, int32_t* gpu_free, int32_t* avail_min,
                     uint32_t* mask);

#ifdef __cplusplus
}
#endif
#endif /* FITGPU_H */
