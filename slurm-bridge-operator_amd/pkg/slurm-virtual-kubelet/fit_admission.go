// fit_admission.go — the call sites of SURVEY.md §8 a10 / b2 / f4: the file a maintainer adds to
// the reference's package pkg/slurm-virtual-kubelet (package slurm_virtual_kubelet, next to
// provider.go and node.go).  Not compiled in this repo's image (no Go toolchain); the C++ side
// it calls (fit_admitter, include/fitgpu.h) is tested on the GPU by tests/test_admit_gpu.py.
//
// What changes, behind the unchanged interfaces (nodeutil.Provider, workload.proto):
//   - CreatePod (provider.go:35-60) asks the engine for a node before SubmitJob.  The 10
//     PodSyncWorkers' concurrent calls are coalesced by fitgpu.Admitter into one fit_place per
//     batch, in pod-creation order.  A pod that does not fit now gets an error, and the library
//     retries it later (the same contract as a failed SubmitJob).
//   - GetPartitionCapacity (node.go:169-199) reports the engine's allocation-aware free capacity
//     instead of the allocation-blind sum (which also adds AlloCpus into the GPU count).
//   - The one-minute timer in NotifyNodeStatus (provider.go:470-488) becomes a ticker that
//     reloads the node table from the agent's Nodes RPC, so placements track Slurm's own state.
package slurm_virtual_kubelet

import (
	"context"
	"fmt"
	"strconv"
	"sync"
	"time"

	"github.com/chriskery/slurm-bridge-operator/pkg/common"
	"github.com/chriskery/slurm-bridge-operator/pkg/fitgpu"
	"github.com/chriskery/slurm-bridge-operator/pkg/workload"
	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/api/resource"
	"k8s.io/klog/v2"
)

// FitAdmission holds the engine of one virtual kubelet (one Slurm partition per VK:
// KubeletServer.SlurmPartition).  The node table is that partition's nodes, in the order of its
// Partition RPC, every node in partition 0.
type FitAdmission struct {
	adm   *fitgpu.Admitter
	eng   *fitgpu.Engine
	mu    sync.Mutex // nodes / names
	names []string   // node id -> Slurm node name
}

// NewFitAdmission creates the engine on GPU `device` and loads the partition's limits and nodes.
func NewFitAdmission(ctx context.Context, vk *SlurmVirtualKubelet, device int) (*FitAdmission, error) {
	eng, err := fitgpu.New(device)
	if err != nil {
		return nil, err // no gfx950 device: the caller keeps the reference behaviour
	}
	res, err := vk.SlurmClient.Resources(ctx, &workload.ResourcesRequest{Partition: vk.KubeletServer.SlurmPartition})
	if err != nil {
		eng.Close()
		return nil, err
	}
	// parseResources' limits after the agent's override merge (pkg/slurm-agent/parse.go:111-190,
	// api/slurm.go:297-341); -1 (UNLIMITED) or an unset 0 → no limit
	limit := func(v int64) int32 {
		if v <= 0 {
			return -1
		}
		return int32(v)
	}
	maxTime := limit(res.WallTime / 60) // seconds → minutes
	if err := eng.LoadPartitions([]int32{maxTime}, []int32{limit(res.CpuPerNode)}, []int32{limit(res.MemPerNode)}); err != nil {
		eng.Close()
		return nil, err
	}
	adm, err := fitgpu.NewAdmitter(eng, 1024, 2*time.Millisecond)
	if err != nil {
		eng.Close()
		return nil, err
	}
	f := &FitAdmission{adm: adm, eng: eng}
	if err := f.Refresh(ctx, vk); err != nil {
		f.Close()
		return nil, err
	}
	return f, nil
}

// Refresh reloads the node table: Partition → Nodes RPCs, free = total − alloc per node
// (workload.proto:165-174).
func (f *FitAdmission) Refresh(ctx context.Context, vk *SlurmVirtualKubelet) error {
	pr, err := vk.SlurmClient.Partition(ctx, &workload.PartitionRequest{Partition: vk.KubeletServer.SlurmPartition})
	if err != nil {
		return err
	}
	nr, err := vk.SlurmClient.Nodes(ctx, &workload.NodesRequest{Nodes: pr.Nodes})
	if err != nil {
		return err
	}
	n := len(nr.Nodes)
	t := fitgpu.Nodes{CPUFree: make([]int32, n), MemFreeMiB: make([]int32, n), GPUFree: make([]int32, n),
		AvailMin: make([]int32, n), PartMask: make([]uint32, n)}
	for i, node := range nr.Nodes {
		t.CPUFree[i] = int32(node.Cpus - node.AlloCpus)
		t.MemFreeMiB[i] = int32(node.Memory - node.AlloMemory)
		t.GPUFree[i] = int32(node.Gpus - node.AlloGpus)
		t.AvailMin[i] = 1<<31 - 1
		t.PartMask[i] = 1
	}
	f.mu.Lock()
	defer f.mu.Unlock()
	if err := f.adm.LoadNodes(t); err != nil {
		return err
	}
	f.names = pr.Nodes
	return nil
}

func (f *FitAdmission) Close() {
	f.adm.Close()
	f.eng.Close()
}

func labelInt(pod *v1.Pod, key string) int64 {
	v, err := strconv.ParseInt(pod.Labels[key], 10, 64)
	if err != nil {
		return 0
	}
	return v
}

// admit places one pod; called by CreatePod before SubmitJob.  nil = the pod has nodes.
func (f *FitAdmission) admit(pod *v1.Pod) error {
	d, err := fitgpu.DemandFromLabels(
		labelInt(pod, common.LabelsResourceRequestNodes), labelInt(pod, common.LabelsResourceRequestCpusPerTask),
		labelInt(pod, common.LabelsResourceRequestMemPerCpu), labelInt(pod, common.LabelsResourceRequestNTasksPerNode),
		labelInt(pod, common.LabelsResourceRequestNTasks), 0, 0, pod.CreationTimestamp.UnixNano())
	if err != nil {
		return err
	}
	a, err := f.adm.Admit(d)
	if err != nil {
		return err
	}
	switch {
	case a.Placed():
		f.mu.Lock()
		names := make([]string, 0, len(a.Nodes))
		for _, id := range a.Nodes {
			if int(id) < len(f.names) {
				names = append(names, f.names[id])
			}
		}
		f.mu.Unlock()
		klog.Infof("pod %s/%s fits on %v (batch %d, %d pods)", pod.Namespace, pod.Name, names, a.Batch, a.BatchJobs)
		return nil
	case a.Nodes[0] == fitgpu.Rejected:
		return fmt.Errorf("pod %s/%s exceeds the partition's limits", pod.Namespace, pod.Name)
	default: // Unplaced: no node has room now; the library retries the pod
		return fmt.Errorf("pod %s/%s: no Slurm node of the partition fits it now", pod.Namespace, pod.Name)
	}
}

// CreatePodWithFit is CreatePod (provider.go:35-60) with the engine's admission in front of
// SubmitJob; provider.go's CreatePod calls it when s.fit != nil:
//
//	if s.fit != nil && needReconcile(pod) {
//	        if err := s.fit.admit(pod); err != nil {
//	                return err
//	        }
//	}
func (s *SlurmVirtualKubeletProvider) CreatePodWithFit(ctx context.Context, pod *v1.Pod, f *FitAdmission) error {
	if needReconcile(pod) {
		if err := s.validateCreatePod(pod); err != nil {
			return err
		}
		if err := f.admit(pod); err != nil {
			return err
		}
	}
	return s.CreatePod(ctx, pod)
}

// PartitionCapacityFromEngine replaces GetPartitionCapacity's sum (node.go:169-199) with the
// engine's free columns after the admitted pods.  Units as the reference: memory quantity in
// bytes from MiB.
func (f *FitAdmission) PartitionCapacityFromEngine() (v1.ResourceList, error) {
	cpu, mem, gpu, err := f.adm.PartitionFree(0)
	if err != nil {
		return nil, err
	}
	rl := v1.ResourceList{}
	rl["cpu"] = *resource.NewQuantity(cpu, resource.DecimalSI)
	rl["memory"] = *resource.NewQuantity(mem<<20, resource.BinarySI)
	if gpu > 0 {
		rl["nvidia.com/gpu"] = *resource.NewQuantity(gpu, resource.DecimalSI)
	}
	rl["pods"] = *resource.NewQuantity(cpu, resource.DecimalSI)
	return rl, nil
}

// RunNodeTicker replaces the one-shot timer of NotifyNodeStatus (provider.go:470-488): every
// period it reloads the node table and publishes the node with the engine's capacity.
func (f *FitAdmission) RunNodeTicker(ctx context.Context, vk *SlurmVirtualKubelet, period time.Duration, nodeFunc func(*v1.Node)) {
	go func() {
		tk := time.NewTicker(period)
		defer tk.Stop()
		for {
			select {
			case <-ctx.Done():
				return
			case <-tk.C:
				if err := f.Refresh(ctx, vk); err != nil {
					klog.Error(err)
					continue
				}
				node, err := vk.NewNodeOrDie()
				if err != nil {
					klog.Error(err)
					continue
				}
				if rl, err := f.PartitionCapacityFromEngine(); err == nil {
					node.Status.Allocatable = rl
				}
				nodeFunc(node)
			}
		}
	}()
}
