"""Command line of the MI355X NanoTel: the flags of NanoTel.R's optparse
block (NanoTel.R:30-93) and its argument checks (NanoTel.R:104-137).

    python -m nanotel_amd -i reads.fastq.gz --save_path out --patterns "TTAGGG"

Multi-GPU: launch one process per GPU with torch.distributed.run; the ranks
index 1/N of the input each, read only their own blocks of chunks and scan
them (driver.py / shard.py); the collectives run over RCCL when every rank has
its own GPU; rank 0 writes the summary.  --use_filter runs the edge pre-filter on the GPU.  --analysis writes
<barcode>_filtered_sorted_summary.csv and <barcode>_results.txt (analysis.py;
not its ggplot2 PNG).  The single-read plots are written as in the reference
(plots.py) unless --no_plots.
"""
import argparse
import os
import sys

from .driver import VERSION, run


def parser():
    ap = argparse.ArgumentParser(prog="nanotel_amd", description="Telomere Analyzer (MI355X hot path)")
    ap.add_argument("-i", "--input_path", default=None, help="Path to input files.( dir or single file)")
    ap.add_argument("--save_path", default=None, help="A path to a directory for storing the output files.")
    ap.add_argument("--format", default="fastq",
                    help='input files format (Either "fastq" (the default) or "fasta", gzip is supported)')
    ap.add_argument("-n", "--nrec", type=int, default=10000,
                    help="The maximum of number of records to read in to memory for each iteration.")
    ap.add_argument("-r", "--rc", action="store_true", help="Should we do reverse complement on the given reads.")
    ap.add_argument("--patterns", default=None, help="Space separated list of pattern(s).")
    ap.add_argument("--min_density", type=float, default=0.6,
                    help="Minimal density to consider a subsequence as a pattern region.")
    ap.add_argument("--subseq_length", type=int, default=100, help="The length of the sub-sequence.")
    ap.add_argument("--use_filter", action="store_true", help="Filter reads accoding to the edge.")
    ap.add_argument("--check_right_edge", action="store_true",
                    help="The expected telomere is at the right edge of the reads.")
    ap.add_argument("--tvr_patterns", default=None,
                    help="Space separated list of additional pattern(s) for Telomere variant repeats.")
    ap.add_argument("--version", action="store_true", help="Print version information and exit")
    ap.add_argument("--analysis", action="store_true",
                    help="Post-processing: filtered sorted summary and results text (no plot).")
    # build-specific
    ap.add_argument("--device", type=int, default=None, help="GPU index (default: LOCAL_RANK or 0)")
    ap.add_argument("--no_reads", action="store_true", help="do not write reads/<serial>.fasta.gz")
    ap.add_argument("--no_plots", action="store_true", help="do not write single_read_plots*/")
    ap.add_argument("--no_jpeg", action="store_true", help="write the .eps plots only")
    ap.add_argument("--legacy_no_ext", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--readr_sci_threshold", type=float, default=None, help=argparse.SUPPRESS)
    return ap


def dist_backend(world, local_world, device_arg, n_gpus, env=os.environ):
    """The process group's backend: NT_DIST_BACKEND when set; otherwise RCCL
    ("nccl") when every local rank has a GPU of its own (the summary-row
    gather and the per-group serial all_reduce then go over xGMI, north_star's
    layout), gloo when ranks share a GPU (an explicit --device, or more local
    ranks than GPUs) or there is one rank."""
    if env.get("NT_DIST_BACKEND"):
        return env["NT_DIST_BACKEND"]
    if world > 1 and device_arg is None and n_gpus >= local_world:
        return "nccl"
    return "gloo"


def main(argv=None):
    a = parser().parse_args(argv)
    if a.version:
        print(VERSION)
        return 0
    if a.patterns is None:
        sys.exit("Error: Missing required parameter:  --patterns")
    if a.save_path is None:
        sys.exit("Error: Missing required parameter:  --save_path")
    if a.input_path is None:
        sys.exit("Error: Missing required parameter:  --input_path")
    if a.format not in ("fasta", "fastq"):
        sys.exit("Error: Format should be a string fastq or fasta")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = a.device if a.device is not None else local
    # NT_DIST_FORCE=1 (with a launcher): join the process group and run the
    # collectives even with one rank -- the RCCL path on a one-GPU box
    grouped = world > 1 or (os.environ.get("NT_DIST_FORCE") == "1" and "WORLD_SIZE" in os.environ)
    if grouped:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        # RCCL when each rank has its own GPU (device tensors for every
        # collective, shard.collective_device), gloo when they share one
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        dist.init_process_group(dist_backend(world, local_world, a.device, torch.cuda.device_count()))
    try:
        run(a.input_path, a.save_path, a.patterns, fmt=a.format, nrec=a.nrec, rc=a.rc,
            min_density=a.min_density, subseq_length=a.subseq_length,
            check_right_edge=a.check_right_edge, tvr_patterns=a.tvr_patterns,
            legacy_no_ext=a.legacy_no_ext, device=dev, write_reads=not a.no_reads,
            sci_threshold=a.readr_sci_threshold, use_filter=a.use_filter,
            analysis=a.analysis, plot=not a.no_plots, plot_jpeg=not a.no_jpeg)
    finally:
        if grouped:
            import torch.distributed as dist
            dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
