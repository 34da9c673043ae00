package fitgpu

/*
#include <stdlib.h>
#include "fitgpu.h"
*/
import "C"

import (
	"fmt"
	"runtime"
	"time"
	"unsafe"
)

// Admitter is the cgo binding of fit_admitter (include/fitgpu.h "batched admission"): the
// coalescer behind CreatePod.  Admit is safe for concurrent use — the virtual kubelet's 10
// PodSyncWorkers (options/options.go:107) call it at once, it blocks while their requests join
// one batch, and the batch is placed by one fit_place in priority order.  While an Admitter owns
// an Engine, use the Engine only through it.
type Admitter struct {
	a   *C.fit_admitter
	eng *Engine // keeps the context alive
}

// Demand of one pod (per node), as fit_pod_demand derives it (PodDemand).
type Demand struct {
	Priority int64 // smaller first: e.g. pod.CreationTimestamp.UnixNano()
	CPU      int32
	MemMiB   int32
	GPU      int32
	WallMin  int32
	Part     uint16 // partition index in LoadPartitions order
	NodesK   uint16 // --nodes (0 = 1, <= MaxK)
	Flags    uint16 // ReqArray: one task of an array job (never pinned to its reserved nodes)
}

// ReqArray marks a request as one task of an array job (FIT_REQ_ARRAY): PodDemand sets it for a
// pod with the array label or an `#SBATCH --array` line; Script then never pins it.
const ReqArray = uint16(C.FIT_REQ_ARRAY)

// Admission is the engine's answer for one request.
type Admission struct {
	Nodes     []int32 // node ids (NodesK of them), or [Unplaced] / [Rejected]
	Batch     int64   // batch the request was placed in
	BatchJobs int32   // requests placed together in that batch
	Order     int32   // this request's position in the batch's placement order
	Ticket    int64   // reservation (> 0 when placed): Confirm once Slurm runs it, Release if not
}

// Placed reports whether the request got its nodes.
func (a Admission) Placed() bool { return len(a.Nodes) > 0 && a.Nodes[0] >= 0 }

// NewAdmitter starts the coalescer: a batch closes maxWait after its first request or at
// maxBatch requests.
func NewAdmitter(e *Engine, maxBatch int, maxWait time.Duration) (*Admitter, error) {
	if e == nil || e.ctx == nil {
		return nil, fmt.Errorf("fitgpu: NewAdmitter on a closed engine")
	}
	var a *C.fit_admitter
	rc := C.fit_admitter_create(e.ctx, C.int32_t(maxBatch), C.int32_t(maxWait.Microseconds()), &a)
	runtime.KeepAlive(e)
	if err := check(rc); err != nil {
		return nil, err
	}
	ad := &Admitter{a: a, eng: e}
	runtime.SetFinalizer(ad, func(ad *Admitter) { ad.Close() })
	return ad, nil
}

func cReq(d Demand) C.fit_admit_req {
	return C.fit_admit_req{
		priority: C.int64_t(d.Priority), cpu: C.int32_t(d.CPU), mem_mib: C.int32_t(d.MemMiB),
		gpu: C.int32_t(d.GPU), wall_min: C.int32_t(d.WallMin), part: C.uint16_t(d.Part),
		nodes_k: C.uint16_t(d.NodesK), flags: C.uint16_t(d.Flags),
	}
}

func goRes(res *C.fit_admit_res, nodesK uint16) Admission {
	k := int(nodesK)
	if k < 1 {
		k = 1
	}
	out := Admission{Batch: int64(res.batch), BatchJobs: int32(res.batch_jobs), Order: int32(res.order),
		Ticket: int64(res.ticket)}
	if res.node[0] < 0 {
		out.Nodes = []int32{int32(res.node[0])}
	} else {
		out.Nodes = make([]int32, k)
		for i := 0; i < k; i++ {
			out.Nodes[i] = int32(res.node[i])
		}
	}
	return out
}

// Admit blocks until the request's batch is placed.
func (ad *Admitter) Admit(d Demand) (Admission, error) {
	if d.NodesK > MaxK {
		return Admission{}, fmt.Errorf("fitgpu: nodes %d > %d", d.NodesK, MaxK)
	}
	req := cReq(d)
	var res C.fit_admit_res
	rc := C.fit_admit(ad.a, &req, &res)
	runtime.KeepAlive(ad) // the finalizer must not destroy the admitter during the blocking call
	if err := check(rc); err != nil {
		return Admission{}, err
	}
	return goRes(&res, d.NodesK), nil
}

// AdmitGroup admits the requests of one pod (PodDemand's tasks) all or nothing, in one batch.
func (ad *Admitter) AdmitGroup(ds []Demand) ([]Admission, error) {
	if len(ds) == 0 {
		return nil, nil
	}
	reqs := make([]C.fit_admit_req, len(ds))
	for i, d := range ds {
		if d.NodesK > MaxK {
			return nil, fmt.Errorf("fitgpu: nodes %d > %d", d.NodesK, MaxK)
		}
		reqs[i] = cReq(d)
	}
	res := make([]C.fit_admit_res, len(ds))
	rc := C.fit_admit_group(ad.a, &reqs[0], C.int32_t(len(ds)), &res[0])
	runtime.KeepAlive(ad)
	if err := check(rc); err != nil {
		return nil, err
	}
	out := make([]Admission, len(ds))
	for i := range ds {
		out[i] = goRes(&res[i], ds[i].NodesK)
	}
	return out, nil
}

// LoadNodes replaces the node table between batches (the node refresh ticker); open reservations
// are taken from the new table again.
func (ad *Admitter) LoadNodes(n Nodes) error {
	cnt := len(n.CPUFree)
	if !sameLen(cnt, len(n.MemFreeMiB), len(n.GPUFree), len(n.AvailMin), len(n.PartMask)) {
		return errLen
	}
	var rc C.int
	if cnt == 0 {
		rc = C.fit_admitter_load_nodes(ad.a, 0, nil, nil, nil, nil, nil)
	} else {
		rc = C.fit_admitter_load_nodes(ad.a, C.int32_t(cnt),
			(*C.int32_t)(&n.CPUFree[0]), (*C.int32_t)(&n.MemFreeMiB[0]), (*C.int32_t)(&n.GPUFree[0]),
			(*C.int32_t)(&n.AvailMin[0]), (*C.uint32_t)(&n.PartMask[0]))
	}
	runtime.KeepAlive(ad)
	return check(rc)
}

// Table flags (fit_node_table.flags).
const (
	// TableState: PartMask carries the nodes' State (IngestNodes: a DOWN / DRAIN node is in no
	// partition), so placements are pinned with --nodelist.
	TableState = int32(C.FIT_TABLE_STATE)
	// TablePin: pin placements on a table without State (the gRPC Nodes RPC's) anyway.
	TablePin = int32(C.FIT_TABLE_PIN)
)

// LoadTable replaces the node table with its node names (NodeNames order: reservations follow
// their node by name across reloads, and Script can pin) and flags (TableState / TablePin).  gen is
// Generation() taken before the table was fetched from Slurm (0 = now): a table fetched before a
// Confirm keeps that reservation, a table older than the loaded one is refused.
func (ad *Admitter) LoadTable(n Nodes, names []string, flags int32, gen int64) error {
	cnt := len(n.CPUFree)
	if !sameLen(cnt, len(n.MemFreeMiB), len(n.GPUFree), len(n.AvailMin), len(n.PartMask)) ||
		(names != nil && len(names) != cnt) {
		return errLen
	}
	t := C.fit_node_table{n: C.int32_t(cnt), flags: C.int32_t(flags), generation: C.int64_t(gen)}
	var pin runtime.Pinner // the struct holds Go pointers during the call (cgo pointer rules)
	defer pin.Unpin()
	if cnt > 0 {
		for _, p := range []*int32{&n.CPUFree[0], &n.MemFreeMiB[0], &n.GPUFree[0], &n.AvailMin[0]} {
			pin.Pin(p)
		}
		pin.Pin(&n.PartMask[0])
		t.cpu_free = (*C.int32_t)(unsafe.Pointer(&n.CPUFree[0]))
		t.mem_free = (*C.int32_t)(unsafe.Pointer(&n.MemFreeMiB[0]))
		t.gpu_free = (*C.int32_t)(unsafe.Pointer(&n.GPUFree[0]))
		t.avail_min = (*C.int32_t)(unsafe.Pointer(&n.AvailMin[0]))
		t.part_mask = (*C.uint32_t)(unsafe.Pointer(&n.PartMask[0]))
	}
	if names != nil {
		cb := C.CBytes(nulJoin(names))
		defer C.free(cb)
		t.names = (*C.char)(cb)
	}
	rc := C.fit_admitter_load_table(ad.a, &t)
	runtime.KeepAlive(ad)
	return check(rc)
}

// Generation hands out a new table generation; take it before the Nodes RPC of a refresh.
func (ad *Admitter) Generation() (int64, error) {
	g := C.fit_admitter_generation(ad.a)
	runtime.KeepAlive(ad)
	if g < 0 {
		return 0, check(C.int(g))
	}
	return int64(g), nil
}

// Script is the sbatch script to submit for a pod admitted with `tickets`: pinned to the
// reserved nodes with `#SBATCH --nodelist=` when the pod is one request on a named table loaded
// with TableState or TablePin (fit_admitter_script), unchanged otherwise.
func (ad *Admitter) Script(tickets []int64, script string) (string, bool, error) {
	if len(tickets) == 0 {
		return script, false, nil
	}
	sc := C.CString(script)
	defer C.free(unsafe.Pointer(sc))
	out := make([]byte, len(script)+64+MaxK*256)
	var pinned C.int32_t
	rc := C.fit_admitter_script(ad.a, (*C.int64_t)(unsafe.Pointer(&tickets[0])), C.int32_t(len(tickets)), sc,
		(*C.char)(unsafe.Pointer(&out[0])), C.int32_t(len(out)), &pinned)
	runtime.KeepAlive(ad)
	if err := check(rc); err != nil {
		return "", false, err
	}
	return string(out[:int(rc)]), pinned != 0, nil
}

// PartitionFree is the allocation-aware free capacity of partition p after the admitted pods.
func (ad *Admitter) PartitionFree(p int) (cpu, memMiB, gpu int64, err error) {
	var c, m, g C.int64_t
	err = check(C.fit_admitter_partition_free(ad.a, C.int32_t(p), &c, &m, &g))
	runtime.KeepAlive(ad)
	return int64(c), int64(m), int64(g), err
}

// Confirm: Slurm now counts the job (it is allocated); the reservation ends at the next LoadNodes.
func (ad *Admitter) Confirm(ticket int64) error {
	err := check(C.fit_admitter_confirm(ad.a, C.int64_t(ticket)))
	runtime.KeepAlive(ad)
	return err
}

// Release: the job will not run (pod deleted, SubmitJob failed); its demand goes back now.
func (ad *Admitter) Release(ticket int64) error {
	err := check(C.fit_admitter_release(ad.a, C.int64_t(ticket)))
	runtime.KeepAlive(ad)
	return err
}

// SetTTL drops an open reservation after `loads` node-table loads (0 = never).
func (ad *Admitter) SetTTL(loads int) error {
	err := check(C.fit_admitter_set_ttl(ad.a, C.int32_t(loads)))
	runtime.KeepAlive(ad)
	return err
}

// Close stops the coalescer; still-queued Admit calls return FIT_E_STATE.
func (ad *Admitter) Close() {
	if ad.a != nil {
		C.fit_admitter_destroy(ad.a)
		ad.a = nil
	}
}
