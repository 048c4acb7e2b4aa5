"""Multi-GPU static plan and the shuffle exchange.

The reference coordinator hands out map tasks (input files) and reduce tasks (partitions) on demand
(src/mr/coordinator.rs:137-215) and the shuffle goes through mr-{m}-{r}.txt files in a shared CWD
(src/mr/worker.rs:117-140, 79-109).  Here the plan is static: rank g maps its shard of the input
files, and owns every partition r with r % G == g.  After the map each rank packs its per-key
records by owner (mrg_job_export), one all-to-all of the per-owner counts tells every rank how much
it receives, and the 24-byte exchange records and the long-key heap bytes follow.  The receiving
rank re-aggregates (mrg_job_import: the same key can arrive from every rank) and reduces its
partitions.  There is exactly one data-path collective, the exchange itself.

Two transports of the same records:
  * library_comm() + Context.shuffle(): the product path, RCCL called from libmrgpu.so
    (mrg_job_shuffle: counts all-to-all, then grouped send/recv over xGMI on the context's stream);
  * shuffle(): export -> torch.distributed all_to_all_single -> import, used with the gloo backend
    (host staged) to rehearse N ranks on one GPU and in the CPU tests.
"""
import torch
import torch.distributed as dist

from . import native

XREC = native.XREC_BYTES

# Per-exchange record of the data all-to-alls (device runs only): start/end events on the current
# stream around the two data collectives, and the bytes this rank sent to / received from peers
# (its own slice stays in HBM).  bench.py turns them into the xGMI roofline fraction.
EXCHANGES = []


def owner_of(partition, n_owners):
    """Static plan: partition r is reduced by rank r % G."""
    return partition % n_owners


def shard_files(n_files, rank, world):
    """Map shard of a rank: files rank, rank + G, ... (equal bytes for equal-size files)."""
    return list(range(rank, n_files, world))


def alltoall_exchange(send_rec, send_heap, rec_counts, heap_counts, group=None, status=0):
    """Exchange per-owner slices.  send_rec: uint8 tensor of sum(rec_counts) * XREC bytes ordered by
    owner; send_heap: uint8 tensor of sum(heap_counts) bytes ordered by owner.  `status` != 0 says this
    rank failed before the exchange: the counts all-to-all carries every rank's status, and every
    rank raises if any failed (no rank is left waiting in the data all-to-alls).
    Returns (recv_rec, recv_heap, recv_rec_counts, recv_heap_counts), ordered by sender."""
    world = dist.get_world_size(group)
    dev = send_rec.device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        # gloo moves host tensors only: stage through host memory (rehearsal of N > 1 on one GPU;
        # the product path is RCCL, which exchanges device buffers directly)
        rr, rh, r_rec, r_heap = alltoall_exchange(send_rec.cpu(), send_heap.cpu(), rec_counts, heap_counts, group,
                                                  status)
        return rr.to(dev), rh.to(dev), r_rec, r_heap
    counts = torch.tensor(list(rec_counts) + list(heap_counts) + [1 if status else 0] * world, dtype=torch.int64,
                          device=dev)
    # [rec_0..rec_{G-1}, heap_0..heap_{G-1}, status x G] -> per destination (rec_o, heap_o, status) triples
    send_c = counts.view(3, world).t().contiguous().view(-1)
    recv_c = torch.empty_like(send_c)
    dist.all_to_all_single(recv_c, send_c, [3] * world, [3] * world, group=group)
    rc = recv_c.view(world, 3).cpu().tolist()
    failed = [o for o, (_, _, st) in enumerate(rc) if st]
    if failed:
        raise native.MrgError(native.ECOMM, "rank %d of the exchange failed before sending" % failed[0])
    r_rec = [int(a) for a, _, _ in rc]
    r_heap = [int(b) for _, b, _ in rc]
    err = None
    try:  # receive buffers; then every rank agrees that all of them have theirs
        recv_rec = torch.empty(max(sum(r_rec), 1) * XREC, dtype=torch.uint8, device=dev)
        recv_heap = torch.empty(max(sum(r_heap), 1), dtype=torch.uint8, device=dev)
    except RuntimeError as e:
        err = e
    flag = torch.tensor([1 if err else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    if err is not None:
        raise err
    if flag.item():
        raise native.MrgError(native.ECOMM, "another rank of the exchange could not allocate its receive buffers")
    timed = dev.type == "cuda"
    if timed:
        me = dist.get_rank(group)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    dist.all_to_all_single(recv_rec[:sum(r_rec) * XREC], send_rec[:sum(rec_counts) * XREC],
                           [x * XREC for x in r_rec], [x * XREC for x in rec_counts], group=group)
    dist.all_to_all_single(recv_heap[:sum(r_heap)], send_heap[:sum(heap_counts)], r_heap, list(heap_counts),
                           group=group)
    if timed:
        ev1.record()
        peers = [o for o in range(world) if o != me]
        EXCHANGES.append({"start": ev0, "end": ev1,
                          "sent": sum(rec_counts[o] * XREC + heap_counts[o] for o in peers),
                          "received": sum(r_rec[o] * XREC + r_heap[o] for o in peers)})
    return recv_rec, recv_heap, r_rec, r_heap


def library_comm(ctx, group=None):
    """The library's RCCL communicator over the ranks of a torch.distributed group, one rank per GPU:
    rank 0 makes the id (mrg_comm_get_id), a broadcast over the group hands it to the others, every
    rank joins (mrg_comm_init, collective).  Use with ctx.shuffle(comm)."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    obj = [native.comm_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return native.Comm(ctx, obj[0], world, rank)


def shuffle(ctx, world, device, group=None):
    """The exchange step of a device-resident job on every rank (after ctx.map()), through
    torch.distributed.  The context's kernels run on its own stream, torch's buffers and collectives
    on torch's current stream: the current stream is drained before the export writes into torch
    buffers and before the import reads what the collectives wrote (the export itself returns only
    after its kernels are done).  A rank whose export fails still takes part in the counts exchange
    (with a failure status), so every rank raises instead of waiting for it."""
    dev = torch.device(device)
    cuda = dev.type == "cuda"
    err = None
    try:
        rec, heap = ctx.export_sizes(world)
        send_rec = torch.empty(max(sum(rec), 1) * XREC, dtype=torch.uint8, device=dev)
        send_heap = torch.empty(max(sum(heap), 1), dtype=torch.uint8, device=dev)
        if cuda:
            torch.cuda.current_stream(dev).synchronize()
        ctx.export(send_rec.data_ptr(), send_heap.data_ptr())
    except (native.MrgError, RuntimeError) as e:  # RuntimeError: a torch allocation
        err = e
        rec, heap = [0] * world, [0] * world
        send_rec = torch.empty(1, dtype=torch.uint8, device=dev)
        send_heap = torch.empty(1, dtype=torch.uint8, device=dev)
    try:
        recv_rec, recv_heap, r_rec, r_heap = alltoall_exchange(send_rec, send_heap, rec, heap, group,
                                                               status=1 if err else 0)
    except native.MrgError:
        if err is not None:
            raise err
        raise
    if cuda:
        torch.cuda.current_stream(dev).synchronize()
    ctx.import_(recv_rec.data_ptr(), sum(r_rec), recv_heap.data_ptr(), sum(r_heap), r_rec, r_heap)
    return sum(r_rec), sum(r_heap)
