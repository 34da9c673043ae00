package fitgpu

/*
#include "fitgpu.h"
*/
import "C"

import (
	"fmt"
	"runtime"
	"time"
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

// Demand of one pod (per node), as fit_job_demand derives it from the SlurmBridgeJob labels.
type Demand struct {
	Priority int64 // smaller first: e.g. pod.CreationTimestamp.UnixNano()
	CPU      int32
	MemMiB   int32
	GPU      int32
	WallMin  int32
	Part     uint16 // partition index in LoadPartitions order
	NodesK   uint16 // --nodes (0 = 1, <= MaxK)
}

// Admission is the engine's answer for one pod.
type Admission struct {
	Nodes     []int32 // node ids (NodesK of them), or [Unplaced] / [Rejected]
	Batch     int64   // batch the pod was placed in
	BatchJobs int32   // pods placed together in that batch
	Order     int32   // this pod's position in the batch's placement order
}

// Placed reports whether the pod got its nodes.
func (a Admission) Placed() bool { return len(a.Nodes) > 0 && a.Nodes[0] >= 0 }

// NewAdmitter starts the coalescer: a batch closes maxWait after its first request or at
// maxBatch requests.
func NewAdmitter(e *Engine, maxBatch int, maxWait time.Duration) (*Admitter, error) {
	if e == nil || e.ctx == nil {
		return nil, fmt.Errorf("fitgpu: NewAdmitter on a closed engine")
	}
	var a *C.fit_admitter
	if err := check(C.fit_admitter_create(e.ctx, C.int32_t(maxBatch), C.int32_t(maxWait.Microseconds()), &a)); err != nil {
		return nil, err
	}
	ad := &Admitter{a: a, eng: e}
	runtime.SetFinalizer(ad, func(ad *Admitter) { ad.Close() })
	return ad, nil
}

// Admit blocks until the pod's batch is placed.
func (ad *Admitter) Admit(d Demand) (Admission, error) {
	if d.NodesK > MaxK {
		return Admission{}, fmt.Errorf("fitgpu: nodes %d > %d", d.NodesK, MaxK)
	}
	req := C.fit_admit_req{
		priority: C.int64_t(d.Priority), cpu: C.int32_t(d.CPU), mem_mib: C.int32_t(d.MemMiB),
		gpu: C.int32_t(d.GPU), wall_min: C.int32_t(d.WallMin), part: C.uint16_t(d.Part),
		nodes_k: C.uint16_t(d.NodesK),
	}
	var res C.fit_admit_res
	if err := check(C.fit_admit(ad.a, &req, &res)); err != nil {
		return Admission{}, err
	}
	k := int(d.NodesK)
	if k < 1 {
		k = 1
	}
	out := Admission{Batch: int64(res.batch), BatchJobs: int32(res.batch_jobs), Order: int32(res.order)}
	if res.node[0] < 0 {
		out.Nodes = []int32{int32(res.node[0])}
	} else {
		out.Nodes = make([]int32, k)
		for i := 0; i < k; i++ {
			out.Nodes[i] = int32(res.node[i])
		}
	}
	return out, nil
}

// LoadNodes replaces the node table between batches (the node refresh ticker).
func (ad *Admitter) LoadNodes(n Nodes) error {
	cnt := len(n.CPUFree)
	if !sameLen(cnt, len(n.MemFreeMiB), len(n.GPUFree), len(n.AvailMin), len(n.PartMask)) {
		return errLen
	}
	if cnt == 0 {
		return check(C.fit_admitter_load_nodes(ad.a, 0, nil, nil, nil, nil, nil))
	}
	return check(C.fit_admitter_load_nodes(ad.a, C.int32_t(cnt),
		(*C.int32_t)(&n.CPUFree[0]), (*C.int32_t)(&n.MemFreeMiB[0]), (*C.int32_t)(&n.GPUFree[0]),
		(*C.int32_t)(&n.AvailMin[0]), (*C.uint32_t)(&n.PartMask[0])))
}

// PartitionFree is the allocation-aware free capacity of partition p after the admitted pods.
func (ad *Admitter) PartitionFree(p int) (cpu, memMiB, gpu int64, err error) {
	var c, m, g C.int64_t
	err = check(C.fit_admitter_partition_free(ad.a, C.int32_t(p), &c, &m, &g))
	return int64(c), int64(m), int64(g), err
}

// Close stops the coalescer; still-queued Admit calls return FIT_E_STATE.
func (ad *Admitter) Close() {
	if ad.a != nil {
		C.fit_admitter_destroy(ad.a)
		ad.a = nil
	}
}

// DemandFromLabels derives a pod's per-node demand from the sbo.kubecluster.org/* labels that
// newSubmitRequestForPod reads (pkg/slurm-virtual-kubelet/provider.go:62-125,
// pkg/common/labels.go:9-14) through the engine's mirror of the operator's arithmetic
// (fit_apply_spec + fit_job_demand, pkg/slurm-bridge-operator/pod.go:70-162).  Missing labels
// are 0 (the operator's defaults then apply); wallMin comes from the job's --time.
func DemandFromLabels(nodes, cpusPerTask, memPerCPU, nTasksPerNode, nTasks int64, wallMin int32,
	part uint16, priority int64) (Demand, error) {
	var r C.fit_job_resources
	C.fit_apply_spec(&r, C.int64_t(nodes), C.int64_t(cpusPerTask), C.int64_t(memPerCPU),
		C.int64_t(nTasksPerNode), nil, C.int64_t(nTasks))
	var cpu, mem, wall C.int32_t
	var k C.uint16_t
	if err := check(C.fit_job_demand(&r, &cpu, &mem, &wall, &k)); err != nil {
		return Demand{}, err
	}
	return Demand{Priority: priority, CPU: int32(cpu), MemMiB: int32(mem), GPU: 0,
		WallMin: wallMin, Part: part, NodesK: uint16(k)}, nil
}
