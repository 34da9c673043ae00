// Package fitgpu is the cgo binding a slurm-bridge-operator maintainer adds to call the MI355X
// placement engine (libfitgpu.so, C-ABI include/fitgpu.h).  It is not compiled in this repo's
// image (no Go toolchain); INTEGRATION.md shows where it is called from.
package fitgpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../fitgpu -lfitgpu -Wl,-rpath,${SRCDIR}/../../fitgpu
#include <stdlib.h>
#include "fitgpu.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"
)

const (
	Unplaced = -1 // FIT_UNPLACED
	Rejected = -2 // FIT_REJECTED
	MaxK     = 8  // FIT_MAX_K: nodes per job (--nodes) fit_place supports
)

// Error carries a negative FIT_E_* code and the library's detail message.
type Error struct {
	Code   int
	Detail string
}

func (e *Error) Error() string {
	return fmt.Sprintf("fitgpu: %s (%d): %s", C.GoString(C.fit_strerror(C.int(e.Code))), e.Code, e.Detail)
}

// EngineFailure reports whether err is the engine failing rather than a decision about a pod:
// a HIP / RCCL runtime error (a watchdog trip included), an allocation failure, no device, or
// a context out of state.  Callers fall back to the reference path on these (INTEGRATION.md).
func EngineFailure(err error) bool {
	var fe *Error
	if !errors.As(err, &fe) {
		return false
	}
	switch fe.Code {
	case int(C.FIT_E_HIP), int(C.FIT_E_RCCL), int(C.FIT_E_OOM), int(C.FIT_E_NODEV), int(C.FIT_E_STATE):
		return true
	}
	return false
}

// SetWatchdog bounds every device-side wait of the persistent engines (fit_set_watchdog_us);
// us <= 0 restores the default (10 s).
func (e *Engine) SetWatchdog(us int64) error {
	return check(C.fit_set_watchdog_us(e.ctx, C.int64_t(us)))
}

// LockDir is the directory of the per-GPU lock file that serialises persistent launches of
// every engine on a GPU (fit_lock_dir).  shared is false when the library fell back to /tmp: in
// the configurator's deployment each virtual kubelet is its own pod with a private /tmp, so
// engines in other pods on the same GPU would not be arbitrated (INTEGRATION.md item 6).
func LockDir() (dir string, shared bool, err error) {
	buf := make([]byte, 4096)
	rc := C.fit_lock_dir((*C.char)(unsafe.Pointer(&buf[0])), C.int32_t(len(buf)))
	if err := check(rc); err != nil {
		return "", false, err
	}
	return C.GoString((*C.char)(unsafe.Pointer(&buf[0]))), rc == 0, nil
}

func check(rc C.int) error {
	if rc < 0 {
		return &Error{Code: int(rc), Detail: C.GoString(C.fit_last_error())}
	}
	return nil
}

// Engine wraps one fit_ctx (one GPU).  Not safe for concurrent use; the VK provider serialises
// its 10 PodSyncWorkers through a batcher (INTEGRATION.md).
type Engine struct{ ctx *C.fit_ctx }

func New(device int) (*Engine, error) {
	opts := C.fit_opts{device: C.int32_t(device), world: 1}
	var ctx *C.fit_ctx
	if err := check(C.fit_create(&opts, &ctx)); err != nil {
		return nil, err
	}
	e := &Engine{ctx: ctx}
	runtime.SetFinalizer(e, func(e *Engine) { e.Close() })
	return e, nil
}

func (e *Engine) Close() {
	if e.ctx != nil {
		C.fit_destroy(e.ctx)
		e.ctx = nil
	}
}

// Nodes is the node table in Client.Nodes order (pkg/slurm-agent/slurm.go:343-364).
type Nodes struct {
	CPUFree, MemFreeMiB, GPUFree, AvailMin []int32
	PartMask                              []uint32
}

// errLen is returned when the columns of one table differ in length: the library reads every
// column for the same count, so a short slice would be read past its end.
var errLen = errors.New("fitgpu: column slices of different lengths")

func sameLen(n int, cols ...int) bool {
	for _, c := range cols {
		if c != n {
			return false
		}
	}
	return true
}

func (e *Engine) LoadNodes(n Nodes) error {
	cnt := len(n.CPUFree)
	if !sameLen(cnt, len(n.MemFreeMiB), len(n.GPUFree), len(n.AvailMin), len(n.PartMask)) {
		return errLen
	}
	if cnt == 0 {
		return check(C.fit_load_nodes(e.ctx, 0, nil, nil, nil, nil, nil))
	}
	// slices of plain integers: no Go pointers inside, the library copies and does not retain
	rc := C.fit_load_nodes(e.ctx, C.int32_t(cnt),
		(*C.int32_t)(unsafe.Pointer(&n.CPUFree[0])), (*C.int32_t)(unsafe.Pointer(&n.MemFreeMiB[0])),
		(*C.int32_t)(unsafe.Pointer(&n.GPUFree[0])), (*C.int32_t)(unsafe.Pointer(&n.AvailMin[0])),
		(*C.uint32_t)(unsafe.Pointer(&n.PartMask[0])))
	runtime.KeepAlive(e) // the finalizer must not destroy the context during the call
	return check(rc)
}

// LoadPartitions takes parseResources' limits (pkg/slurm-agent/parse.go:111-190), -1 = UNLIMITED.
func (e *Engine) LoadPartitions(maxTimeMin, maxCPUs, maxMemMiB []int32) error {
	p := len(maxTimeMin)
	if !sameLen(p, len(maxCPUs), len(maxMemMiB)) {
		return errLen
	}
	if p == 0 {
		return check(C.fit_load_partitions(e.ctx, 0, nil, nil, nil))
	}
	return check(C.fit_load_partitions(e.ctx, C.int32_t(p), (*C.int32_t)(unsafe.Pointer(&maxTimeMin[0])),
		(*C.int32_t)(unsafe.Pointer(&maxCPUs[0])), (*C.int32_t)(unsafe.Pointer(&maxMemMiB[0]))))
}

// Jobs in priority order, per-node demand (DESIGN.md §2).
type Jobs struct {
	CPU, MemMiB, GPU, WallMin []int32
	Part, NodesK              []uint16
}

type Stats = C.fit_stats

// Place returns node ids (or Unplaced / Rejected) per job, kmax entries per job.
// NodesK may be empty (every job takes one node); otherwise it has one entry per job.
func (e *Engine) Place(j Jobs, kmax int) ([]int32, Stats, error) {
	cnt := len(j.CPU)
	var st C.fit_stats
	if kmax < 1 || kmax > MaxK {
		return nil, st, fmt.Errorf("fitgpu: kmax %d outside [1, %d]", kmax, MaxK)
	}
	if !sameLen(cnt, len(j.MemMiB), len(j.GPU), len(j.WallMin), len(j.Part)) ||
		(len(j.NodesK) != 0 && len(j.NodesK) != cnt) {
		return nil, st, errLen
	}
	out := make([]int32, cnt*kmax)
	if cnt == 0 {
		return out, st, nil
	}
	var nk *C.uint16_t // NULL: every job takes one node
	if len(j.NodesK) > 0 {
		nk = (*C.uint16_t)(unsafe.Pointer(&j.NodesK[0]))
	}
	rc := C.fit_place(e.ctx, C.int32_t(cnt), (*C.int32_t)(unsafe.Pointer(&j.CPU[0])),
		(*C.int32_t)(unsafe.Pointer(&j.MemMiB[0])), (*C.int32_t)(unsafe.Pointer(&j.GPU[0])),
		(*C.int32_t)(unsafe.Pointer(&j.WallMin[0])), (*C.uint16_t)(unsafe.Pointer(&j.Part[0])),
		nk, C.int32_t(kmax), (*C.int32_t)(unsafe.Pointer(&out[0])), &st)
	runtime.KeepAlive(e)
	return out, st, check(rc)
}

// PartitionFree is the allocation-aware replacement for GetPartitionCapacity's sum
// (pkg/slurm-virtual-kubelet/node.go:183-190).
func (e *Engine) PartitionFree(p int) (cpu, memMiB, gpu int64, err error) {
	var c, m, g C.int64_t
	err = check(C.fit_partition_free(e.ctx, C.int32_t(p), &c, &m, &g))
	runtime.KeepAlive(e)
	return int64(c), int64(m), int64(g), err
}

// Releases are the end times of the jobs already running on each node (squeue EndTime), CSR by
// node id: node x's events are [Off[x], Off[x+1]) with non-decreasing Slot (DESIGN.md §2b).
type Releases struct {
	Off, Slot, CPU, MemMiB, GPU []int32
}

// LoadTimeline builds the backfill horizon (slots of slotMin minutes, <= 1024 slots) on top of
// the node table of the last LoadNodes.
func (e *Engine) LoadTimeline(slots, slotMin int, r Releases) error {
	if !sameLen(len(r.Slot), len(r.CPU), len(r.MemMiB), len(r.GPU)) {
		return errLen
	}
	if len(r.Off) > 0 && int(r.Off[len(r.Off)-1]) > len(r.Slot) {
		return fmt.Errorf("fitgpu: Off ends at %d but there are %d release events", r.Off[len(r.Off)-1], len(r.Slot))
	}
	if len(r.Off) == 0 {
		return check(C.fit_load_timeline(e.ctx, C.int32_t(slots), C.int32_t(slotMin), nil, nil, nil, nil, nil))
	}
	var s, c, m, g *C.int32_t
	if len(r.Slot) > 0 {
		s, c = (*C.int32_t)(unsafe.Pointer(&r.Slot[0])), (*C.int32_t)(unsafe.Pointer(&r.CPU[0]))
		m, g = (*C.int32_t)(unsafe.Pointer(&r.MemMiB[0])), (*C.int32_t)(unsafe.Pointer(&r.GPU[0]))
	}
	return check(C.fit_load_timeline(e.ctx, C.int32_t(slots), C.int32_t(slotMin),
		(*C.int32_t)(unsafe.Pointer(&r.Off[0])), s, c, m, g))
}

// RunningJob is one job the caller knows is running (the virtual kubelet's own pods): its engine
// node rows (JobInfo.node_list expanded with ExpandHostlist, mapped through the NodeNames table),
// the minutes left until JobInfo.end_time (workload.proto:252-292) and its per-node demand.
type RunningJob struct {
	Nodes            []int32
	MinutesLeft      int64
	CPU, MemMiB, GPU int32
}

// ReleaseEvents turns running jobs into the release events LoadTimeline reads
// (fit_release_events): each job hands its demand back on each of its nodes at slot
// max(1, ceil(MinutesLeft / slotMin)), capped at the horizon.
func ReleaseEvents(nodes int, jobs []RunningJob, slots, slotMin int) (Releases, error) {
	off := make([]int32, len(jobs)+1)
	var rows []int32
	rem := make([]int64, len(jobs))
	cpu, mem, gpu := make([]int32, len(jobs)), make([]int32, len(jobs)), make([]int32, len(jobs))
	for i, j := range jobs {
		rows = append(rows, j.Nodes...)
		off[i+1] = int32(len(rows))
		rem[i], cpu[i], mem[i], gpu[i] = j.MinutesLeft, j.CPU, j.MemMiB, j.GPU
	}
	e := len(rows)
	r := Releases{Off: make([]int32, nodes+1), Slot: make([]int32, e), CPU: make([]int32, e),
		MemMiB: make([]int32, e), GPU: make([]int32, e)}
	p32 := func(v []int32) *C.int32_t {
		if len(v) == 0 {
			return nil
		}
		return (*C.int32_t)(unsafe.Pointer(&v[0]))
	}
	var remp *C.int64_t
	if len(rem) > 0 {
		remp = (*C.int64_t)(unsafe.Pointer(&rem[0]))
	}
	n := C.fit_release_events(C.int32_t(nodes), C.int32_t(len(jobs)), p32(off), p32(rows), remp, p32(cpu),
		p32(mem), p32(gpu), C.int32_t(slots), C.int32_t(slotMin), p32(r.Off), p32(r.Slot), p32(r.CPU),
		p32(r.MemMiB), p32(r.GPU), C.int32_t(e))
	runtime.KeepAlive(rows)
	if err := check(n); err != nil {
		return Releases{}, err
	}
	return r, nil
}

// PlaceBackfill gives each job (one node) its node and earliest start slot (DESIGN.md §2b);
// node is Unplaced when nothing fits inside the horizon, Rejected for partition limits.
func (e *Engine) PlaceBackfill(j Jobs) (node, start []int32, st Stats, err error) {
	cnt := len(j.CPU)
	if !sameLen(cnt, len(j.MemMiB), len(j.GPU), len(j.WallMin), len(j.Part)) {
		return nil, nil, st, errLen
	}
	node, start = make([]int32, cnt), make([]int32, cnt)
	if cnt == 0 {
		return node, start, st, nil
	}
	rc := C.fit_place_tl(e.ctx, C.int32_t(cnt), (*C.int32_t)(unsafe.Pointer(&j.CPU[0])),
		(*C.int32_t)(unsafe.Pointer(&j.MemMiB[0])), (*C.int32_t)(unsafe.Pointer(&j.GPU[0])),
		(*C.int32_t)(unsafe.Pointer(&j.WallMin[0])), (*C.uint16_t)(unsafe.Pointer(&j.Part[0])),
		(*C.int32_t)(unsafe.Pointer(&node[0])), (*C.int32_t)(unsafe.Pointer(&start[0])), &st)
	runtime.KeepAlive(e)
	return node, start, st, check(rc)
}

// IngestNodes turns `scontrol show nodes` output into the engine's node table (Client.Nodes +
// parseNode, pkg/slurm-agent/slurm.go:354-363 / parse.go:291-308, plus Gres/GresUsed, State,
// Partitions and NodeName), partitions[p] = the partition of part_mask bit p.
func IngestNodes(text string, partitions []string) (Nodes, []string, error) {
	ct := C.CString(text)
	defer C.free(unsafe.Pointer(ct))
	blob := make([]byte, 0, 64)
	for _, p := range partitions {
		blob = append(append(blob, p...), 0)
	}
	blob = append(blob, 0)
	cp := C.CBytes(blob)
	defer C.free(cp)
	capn := 2
	for i := 0; i+1 < len(text); i++ {
		if text[i] == '\n' && text[i+1] == '\n' {
			capn++
		}
	}
	n := Nodes{make([]int32, capn), make([]int32, capn), make([]int32, capn), make([]int32, capn),
		make([]uint32, capn)}
	names := make([]byte, len(text)+64)
	rc := C.fit_ingest_nodes(ct, (*C.char)(cp), C.int32_t(len(partitions)), C.int32_t(capn),
		(*C.int32_t)(unsafe.Pointer(&n.CPUFree[0])), (*C.int32_t)(unsafe.Pointer(&n.MemFreeMiB[0])),
		(*C.int32_t)(unsafe.Pointer(&n.GPUFree[0])), (*C.int32_t)(unsafe.Pointer(&n.AvailMin[0])),
		(*C.uint32_t)(unsafe.Pointer(&n.PartMask[0])), (*C.char)(unsafe.Pointer(&names[0])),
		C.int32_t(len(names)))
	if err := check(rc); err != nil {
		return Nodes{}, nil, err
	}
	cnt := int(rc)
	n = Nodes{n.CPUFree[:cnt], n.MemFreeMiB[:cnt], n.GPUFree[:cnt], n.AvailMin[:cnt], n.PartMask[:cnt]}
	out := make([]string, 0, cnt)
	for i, b := 0, 0; i < len(names) && len(out) < cnt; i++ {
		if names[i] == 0 {
			out = append(out, string(names[b:i]))
			b = i + 1
		}
	}
	return n, out, nil
}

// ---- CreatePod call site (include/fitgpu.h): every rule is in C; Go only marshals strings --------

// PodLabels holds the sbo.kubecluster.org/<key> label values newSubmitRequestForPod reads
// (pkg/slurm-virtual-kubelet/provider.go:74-123, keys pkg/common/labels.go:9-14); nil = absent.
type PodLabels struct {
	Nodes, CpusPerTask, MemPerCpu, NtasksPerNode, Array, Ntasks *string
}

func cstr(s *string) *C.char {
	if s == nil {
		return nil
	}
	return C.CString(*s)
}

// PodDemand derives a pod's admission requests from its labels and sbatch script (fit_pod_demand):
// the script's #SBATCH header under the labels, the operator's defaults, one request per array
// task that may run at once.
func PodDemand(l PodLabels, script string, part uint16, priority int64) ([]Demand, error) {
	fields := []*string{l.Nodes, l.CpusPerTask, l.MemPerCpu, l.NtasksPerNode, l.Array, l.Ntasks}
	cs := make([]*C.char, len(fields))
	for i, f := range fields {
		cs[i] = cstr(f)
		if cs[i] != nil {
			defer C.free(unsafe.Pointer(cs[i]))
		}
	}
	lab := C.fit_pod_labels{nodes: cs[0], cpus_per_task: cs[1], mem_per_cpu: cs[2],
		ntasks_per_node: cs[3], array: cs[4], ntasks: cs[5]}
	sc := C.CString(script)
	defer C.free(unsafe.Pointer(sc))
	n := C.fit_pod_demand(&lab, sc, C.uint16_t(part), C.int64_t(priority), nil, 0)
	if err := check(n); err != nil {
		return nil, err
	}
	reqs := make([]C.fit_admit_req, int(n))
	if err := check(C.fit_pod_demand(&lab, sc, C.uint16_t(part), C.int64_t(priority), &reqs[0], n)); err != nil {
		return nil, err
	}
	out := make([]Demand, len(reqs))
	for i, r := range reqs {
		out[i] = Demand{Priority: int64(r.priority), CPU: int32(r.cpu), MemMiB: int32(r.mem_mib),
			GPU: int32(r.gpu), WallMin: int32(r.wall_min), Part: uint16(r.part), NodesK: uint16(r.nodes_k),
			Flags: uint16(r.flags)}
	}
	return out, nil
}

// ScriptWithNodelist forwards the engine's nodes to slurmctld: the script with
// `#SBATCH --nodelist=` at the end of its #SBATCH header (fit_script_with_nodelist).
func ScriptWithNodelist(script string, names []string, nodes []int32) (string, error) {
	if len(nodes) == 0 {
		return script, nil
	}
	blob := nulJoin(names)
	cb := C.CBytes(blob)
	defer C.free(cb)
	sc := C.CString(script)
	defer C.free(unsafe.Pointer(sc))
	out := make([]byte, len(script)+32+len(blob)+1)
	rc := C.fit_script_with_nodelist(sc, (*C.char)(cb), C.int32_t(len(names)),
		(*C.int32_t)(unsafe.Pointer(&nodes[0])), C.int32_t(len(nodes)),
		(*C.char)(unsafe.Pointer(&out[0])), C.int32_t(len(out)))
	if err := check(rc); err != nil {
		return "", err
	}
	return string(out[:int(rc)]), nil
}

func nulJoin(names []string) []byte {
	blob := make([]byte, 0, 16*len(names)+1)
	for _, nm := range names {
		blob = append(append(blob, nm...), 0)
	}
	return append(blob, 0)
}

// NodeNames expands the Partition RPC's node list (parsePartition splits `Nodes=` on every comma,
// pkg/slurm-agent/parse.go:278-289) into the node names to send to the Nodes RPC: one engine row
// per name, record i of the answer is name i (fit_node_names).
func NodeNames(entries []string) ([]string, error) {
	if len(entries) == 0 {
		return []string{}, nil
	}
	cb := C.CBytes(nulJoin(entries))
	defer C.free(cb)
	for size := 1 << 16; ; size *= 16 {
		buf := make([]byte, size)
		n := C.fit_node_names((*C.char)(cb), C.int32_t(len(entries)), (*C.char)(unsafe.Pointer(&buf[0])),
			C.int32_t(size))
		if n == C.FIT_E_INVAL && size < 1<<24 {
			continue // buffer too small (a repeated name is FIT_E_PARSE: reported at once)
		}
		if err := check(n); err != nil {
			return nil, err
		}
		out := make([]string, 0, int(n))
		for b, i := 0, 0; len(out) < int(n); i++ {
			if buf[i] == 0 {
				out = append(out, string(buf[b:i]))
				b = i + 1
			}
		}
		return out, nil
	}
}

// SetMaxArraySize sets Slurm's MaxArraySize for PodDemand (process-wide); returns the previous value.
func SetMaxArraySize(n int32) (int32, error) {
	rc := C.fit_set_max_array_size(C.int32_t(n))
	if rc < 0 {
		return 0, check(C.int(rc))
	}
	return int32(rc), nil
}

// PartitionLimits converts a ResourcesResponse (workload.proto:137-148) into LoadPartitions' limits.
func PartitionLimits(wallTimeS, cpuPerNode, memPerNode int64) (maxTimeMin, maxCPUs, maxMemMiB int32, err error) {
	var t, c, m C.int32_t
	err = check(C.fit_partition_limits(C.int64_t(wallTimeS), C.int64_t(cpuPerNode), C.int64_t(memPerNode), &t, &c, &m))
	return int32(t), int32(c), int32(m), err
}

// ProtoNode is one workload.Node (workload.proto:165-174).
type ProtoNode struct {
	Cpus, Memory, Gpus, AlloCpus, AlloMemory, AlloGpus int64
}

// NodeColumns turns NodesResponse rows into a node table (free = total − alloc), every node in
// the partitions of partMask.
func NodeColumns(nodes []ProtoNode, partMask uint32) (Nodes, error) {
	n := len(nodes)
	t := Nodes{make([]int32, n), make([]int32, n), make([]int32, n), make([]int32, n), make([]uint32, n)}
	if n == 0 {
		return t, nil
	}
	rows := make([]C.fit_node, n)
	for i, x := range nodes {
		rows[i] = C.fit_node{cpus: C.int64_t(x.Cpus), memory: C.int64_t(x.Memory), gpus: C.int64_t(x.Gpus),
			allo_cpus: C.int64_t(x.AlloCpus), allo_memory: C.int64_t(x.AlloMemory), allo_gpus: C.int64_t(x.AlloGpus)}
	}
	rc := C.fit_node_columns(&rows[0], C.int32_t(n), C.uint32_t(partMask),
		(*C.int32_t)(unsafe.Pointer(&t.CPUFree[0])), (*C.int32_t)(unsafe.Pointer(&t.MemFreeMiB[0])),
		(*C.int32_t)(unsafe.Pointer(&t.GPUFree[0])), (*C.int32_t)(unsafe.Pointer(&t.AvailMin[0])),
		(*C.uint32_t)(unsafe.Pointer(&t.PartMask[0])))
	return t, check(rc)
}
