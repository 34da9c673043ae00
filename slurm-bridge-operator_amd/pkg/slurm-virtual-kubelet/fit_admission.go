// fit_admission.go — the call sites of SURVEY.md §8 a10 / b2 / f4: the file a maintainer adds to
// the reference's package pkg/slurm-virtual-kubelet (package slurm_virtual_kubelet, next to
// provider.go and node.go).  Not compiled in this repo's image (no Go toolchain).  It holds no
// rule of its own: labels and script go to fit_pod_demand, the decision comes back through
// fit_script_with_nodelist, limits and node rows through fit_partition_limits / fit_node_columns
// (include/fitgpu.h "CreatePod call site") — all of which the tests call (tests/test_callsite.py,
// tests/test_admit_gpu.py).
//
// What changes, behind the unchanged interfaces (nodeutil.Provider, workload.proto):
//   - CreatePod (provider.go:35-60) asks the engine for nodes before SubmitJob.  The 10
//     PodSyncWorkers' concurrent calls are coalesced by fitgpu.Admitter into one fit_place per
//     batch, in pod-creation order; an array job's tasks are admitted all or nothing.  A pod that
//     does not fit now gets an error, and the library retries it later (the same contract as a
//     failed SubmitJob).  A placed pod's script carries `#SBATCH --nodelist=` so slurmctld runs it
//     where the engine reserved it (SubmitJobRequest.script, workload.proto:66).
//   - The reservation lives until the pod's job runs (Confirm, from the status poll) or the pod is
//     deleted / its submission fails (Release); node-table reloads re-apply open reservations.
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

	"github.com/chriskery/slurm-bridge-operator/apis/kubecluster.org/v1alpha1"
	"github.com/chriskery/slurm-bridge-operator/pkg/common"
	"github.com/chriskery/slurm-bridge-operator/pkg/fitgpu"
	"github.com/chriskery/slurm-bridge-operator/pkg/workload"
	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/api/resource"
	"k8s.io/apimachinery/pkg/types"
	"k8s.io/klog/v2"
)

// FitAdmission holds the engine of one virtual kubelet (one Slurm partition per VK:
// KubeletServer.SlurmPartition, pkg/configurator/configurator.go:151-171).  The node table is that
// partition's nodes, one row per name of its expanded Partition RPC list, every node in partition 0.
type FitAdmission struct {
	adm     *fitgpu.Admitter
	eng     *fitgpu.Engine
	mu      sync.Mutex            // tickets
	tickets map[types.UID][]int64 // open reservations per pod
	// PinWithoutState: forward the engine's nodes with --nodelist although the gRPC node table has
	// no node State (workload.proto:165-174) — a pod pinned to a DOWN / DRAIN node then pends in
	// Slurm while its reservation holds the capacity.  Default false: the engine gates capacity and
	// slurmctld picks the nodes.
	PinWithoutState bool
}

// NewFitAdmission creates the engine on GPU `device` and loads the partition's limits and nodes;
// pinWithoutState sets FitAdmission.PinWithoutState.
func NewFitAdmission(ctx context.Context, vk *SlurmVirtualKubelet, device int, pinWithoutState bool) (*FitAdmission, error) {
	eng, err := fitgpu.New(device)
	if err != nil {
		return nil, err // no gfx950 device: the caller keeps the reference behaviour
	}
	// the device lock must be a host path every VK pod of this host mounts (INTEGRATION.md item 6)
	if dir, shared, err := fitgpu.LockDir(); err == nil && !shared {
		klog.Warningf("fit: device lock in %s (no FIT_LOCK_DIR, no /var/run/fitgpu): engines in other "+
			"virtual-kubelet pods on this GPU are not arbitrated; mount a hostPath at /var/run/fitgpu", dir)
	}
	res, err := vk.SlurmClient.Resources(ctx, &workload.ResourcesRequest{Partition: vk.KubeletServer.SlurmPartition})
	if err != nil {
		eng.Close()
		return nil, err
	}
	// parseResources' limits after the agent's override merge (pkg/slurm-agent/parse.go:111-190,
	// api/slurm.go:297-341), converted by fit_partition_limits
	maxTime, maxCPUs, maxMem, err := fitgpu.PartitionLimits(res.WallTime, res.CpuPerNode, res.MemPerNode)
	if err == nil {
		err = eng.LoadPartitions([]int32{maxTime}, []int32{maxCPUs}, []int32{maxMem})
	}
	if err != nil {
		eng.Close()
		return nil, err
	}
	adm, err := fitgpu.NewAdmitter(eng, 1024, 2*time.Millisecond)
	if err != nil {
		eng.Close()
		return nil, err
	}
	f := &FitAdmission{adm: adm, eng: eng, tickets: map[types.UID][]int64{}, PinWithoutState: pinWithoutState}
	if err := f.Refresh(ctx, vk); err != nil {
		f.Close()
		return nil, err
	}
	return f, nil
}

// Refresh reloads the node table: Partition RPC → fit_node_names (the hostlist parsePartition
// leaves unexpanded, pkg/slurm-agent/parse.go:278-289) → Nodes RPC for exactly those names →
// fit_node_columns (free = total − alloc per node, workload.proto:165-174).  Client.Nodes joins the
// names for one `scontrol show nodes` and returns its records in output order
// (pkg/slurm-agent/slurm.go:343-364): record i is taken to be name i, and a reply with another
// record count is refused.  The generation is taken before the RPC, so a confirmation that lands
// while it is in flight keeps its reservation (the reply does not count that job yet).  Open
// reservations follow their node by name (fit_admitter_load_table).
func (f *FitAdmission) Refresh(ctx context.Context, vk *SlurmVirtualKubelet) error {
	gen, err := f.adm.Generation()
	if err != nil {
		return err
	}
	pr, err := vk.SlurmClient.Partition(ctx, &workload.PartitionRequest{Partition: vk.KubeletServer.SlurmPartition})
	if err != nil {
		return err
	}
	names, err := fitgpu.NodeNames(pr.Nodes)
	if err != nil {
		return err
	}
	nr, err := vk.SlurmClient.Nodes(ctx, &workload.NodesRequest{Nodes: names})
	if err != nil {
		return err
	}
	if len(nr.Nodes) != len(names) {
		return fmt.Errorf("fit: partition %s lists %d nodes, scontrol returned %d records",
			vk.KubeletServer.SlurmPartition, len(names), len(nr.Nodes))
	}
	rows := make([]fitgpu.ProtoNode, len(nr.Nodes))
	for i, n := range nr.Nodes {
		rows[i] = fitgpu.ProtoNode{Cpus: n.Cpus, Memory: n.Memory, Gpus: n.Gpus,
			AlloCpus: n.AlloCpus, AlloMemory: n.AlloMemory, AlloGpus: n.AlloGpus}
	}
	t, err := fitgpu.NodeColumns(rows, 1)
	if err != nil {
		return err
	}
	flags := int32(0) // no State on this path: capacity gate unless the operator pins anyway
	if f.PinWithoutState {
		flags = fitgpu.TablePin
	}
	return f.adm.LoadTable(t, names, flags, gen)
}

func (f *FitAdmission) Close() {
	f.adm.Close()
	f.eng.Close()
}

func podLabels(pod *v1.Pod) fitgpu.PodLabels {
	get := func(k string) *string {
		if v, ok := pod.Labels[k]; ok {
			return &v
		}
		return nil
	}
	return fitgpu.PodLabels{
		Nodes: get(common.LabelsResourceRequestNodes), CpusPerTask: get(common.LabelsResourceRequestCpusPerTask),
		MemPerCpu: get(common.LabelsResourceRequestMemPerCpu), NtasksPerNode: get(common.LabelsResourceRequestNTasksPerNode),
		Array: get(common.LabelsResourceRequestArray), Ntasks: get(common.LabelsResourceRequestNTasks),
	}
}

// admit places one pod; called by CreatePodWithFit before SubmitJob.  Returns the script to
// submit (with the engine's nodes for a non-array job) and the pod's reservations.
func (f *FitAdmission) admit(pod *v1.Pod) (string, []int64, error) {
	script := pod.Spec.Containers[0].Command[0] // validateCreatePod checked the shape
	ds, err := fitgpu.PodDemand(podLabels(pod), script, 0, pod.CreationTimestamp.UnixNano())
	if err != nil {
		return "", nil, err
	}
	as, err := f.adm.AdmitGroup(ds)
	if err != nil {
		return "", nil, err
	}
	switch {
	case as[0].Placed(): // all or nothing: every task has its nodes
		tickets := make([]int64, len(as))
		for i, a := range as {
			tickets[i] = a.Ticket
		}
		// pinned to the reserved nodes when the table allows it (one request, named table with
		// State or PinWithoutState); an array job's tasks share one sbatch and stay unpinned
		out, pinned, err := f.adm.Script(tickets, script)
		if err != nil {
			f.release(tickets)
			return "", nil, err
		}
		klog.Infof("pod %s/%s fits on %v (batch %d, %d requests, pinned %v)", pod.Namespace, pod.Name,
			as[0].Nodes, as[0].Batch, as[0].BatchJobs, pinned)
		return out, tickets, nil
	case as[0].Nodes[0] == fitgpu.Rejected:
		return "", nil, fmt.Errorf("pod %s/%s exceeds the partition's limits", pod.Namespace, pod.Name)
	default: // Unplaced: no node has room now; the library retries the pod
		return "", nil, fmt.Errorf("pod %s/%s: no Slurm node of the partition fits it now", pod.Namespace, pod.Name)
	}
}

func (f *FitAdmission) release(tickets []int64) {
	for _, t := range tickets {
		if err := f.adm.Release(t); err != nil {
			klog.Error(err)
		}
	}
}

// CreatePodWithFit is CreatePod (provider.go:35-60) with the engine's admission in front of
// SubmitJob and its nodes in the submitted script; provider.go's CreatePod delegates to it when
// s.fit != nil and needReconcile(pod).  An engine failure (fitgpu.EngineFailure) falls back to the
// reference submission: unpinned, no reservation, logged.
func (s *SlurmVirtualKubeletProvider) CreatePodWithFit(ctx context.Context, pod *v1.Pod, f *FitAdmission) error {
	if !needReconcile(pod) {
		return s.CreatePod(ctx, pod)
	}
	if err := s.validateCreatePod(pod); err != nil {
		return err
	}
	script, tickets, err := f.admit(pod)
	if err != nil {
		if !fitgpu.EngineFailure(err) {
			return err // a decision (no room now, over the partition's limits) or a bad pod
		}
		// the engine failed (a HIP error, a watchdog trip, no device): the pod goes the reference
		// way instead of being retried against an engine that cannot answer — submitted as
		// CreatePod submits it (provider.go:35-60): its own script, unpinned, no reservation
		klog.Errorf("fit: engine failure admitting pod %s/%s, submitting it without a fit check: %v",
			pod.Namespace, pod.Name, err)
		script, tickets = pod.Spec.Containers[0].Command[0], nil
	}
	submitRequest := s.newSubmitRequestForPod(pod)
	submitRequest.Script = script
	submitJobResp, err := s.vk.SlurmClient.SubmitJob(ctx, submitRequest)
	if err != nil {
		f.release(tickets) // the job will not run: its capacity goes back
		return err
	}
	f.mu.Lock()
	f.tickets[pod.UID] = tickets
	f.mu.Unlock()
	s.vk.recorder.Eventf(pod, v1.EventTypeNormal, common.NewReason(v1alpha1.SlurmBridgeJobKind, common.SlurmBridgeJobCreatedReason),
		"SlurmBridgeJob submit to the slurm-agent %s, job id is %d", s.vk.KubeletServer.AgentEndpoint, submitJobResp.JobId)
	s.knownPods.Store(pod.UID, strconv.FormatInt(submitJobResp.GetJobId(), 10))
	s.addAndUpdateSlurmJobInfo(pod, strconv.FormatInt(submitJobResp.GetJobId(), 10))
	return nil
}

// ConfirmRunning is called from GetPodStatus (provider.go:195) once the pod's job has left the
// pending state: Slurm counts its allocation from now on, so the reservation ends at the next
// Refresh instead of being re-applied.
func (f *FitAdmission) ConfirmRunning(pod *v1.Pod, phase v1.PodPhase) {
	if phase == v1.PodPending {
		return
	}
	f.mu.Lock()
	tickets := f.tickets[pod.UID]
	delete(f.tickets, pod.UID)
	f.mu.Unlock()
	for _, t := range tickets {
		if err := f.adm.Confirm(t); err != nil {
			klog.Error(err)
		}
	}
}

// DeletePodWithFit is DeletePod (provider.go:156-181) plus the release of a reservation the pod
// still holds (deleted before its job ran).
func (s *SlurmVirtualKubeletProvider) DeletePodWithFit(ctx context.Context, pod *v1.Pod, f *FitAdmission) error {
	f.mu.Lock()
	tickets := f.tickets[pod.UID]
	delete(f.tickets, pod.UID)
	f.mu.Unlock()
	f.release(tickets)
	return s.DeletePod(ctx, pod)
}

// PartitionCapacityFromEngine replaces GetPartitionCapacity's sum (node.go:169-199) with the
// engine's free columns after the admitted pods.  Memory is reported as MiB << 20 bytes — a
// deliberate departure from the reference's mem*(2<<10) (node.go:193, MiB × 2048), which matches
// neither the node's MiB nor the pods' KiB-as-bytes requests (pod.go:160).
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
