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
	return check(C.fit_load_nodes(e.ctx, C.int32_t(cnt),
		(*C.int32_t)(unsafe.Pointer(&n.CPUFree[0])), (*C.int32_t)(unsafe.Pointer(&n.MemFreeMiB[0])),
		(*C.int32_t)(unsafe.Pointer(&n.GPUFree[0])), (*C.int32_t)(unsafe.Pointer(&n.AvailMin[0])),
		(*C.uint32_t)(unsafe.Pointer(&n.PartMask[0]))))
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
	return out, st, check(rc)
}

// PartitionFree is the allocation-aware replacement for GetPartitionCapacity's sum
// (pkg/slurm-virtual-kubelet/node.go:183-190).
func (e *Engine) PartitionFree(p int) (cpu, memMiB, gpu int64, err error) {
	var c, m, g C.int64_t
	err = check(C.fit_partition_free(e.ctx, C.int32_t(p), &c, &m, &g))
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
