"""The CLI's options (find_circ.py:383-413), in a module that imports nothing but optparse: the
prestart (prestart.py) parses the command line with them before numpy is imported."""
import optparse

USAGE = """
   bwa mem -t<threads> [-p] -A2 -B10 -k 15 -T 1 $GENOME_INDEX reads.fastq.gz | %prog [options]

   OR:

   %prog [options] <bwa_mem_genome_alignments.bam>
"""


def build_parser(parser_class=optparse.OptionParser) -> optparse.OptionParser:
    p = parser_class(usage=USAGE)
    a = p.add_option
    a("-v", "--version", dest="version", action="store_true", default=False, help="get version information")
    a("-S", "--system", dest="system", type=str, default="", help="model system database (needs byo; unsupported)")
    a("-G", "--genome", dest="genome", type=str, default="", help="path to genome (one multichromosome FASTA file)")
    a("", "--known-circ", dest="known_circ", type=str, default="", help="file with known circRNA junctions (BED6)")
    a("", "--known-lin", dest="known_lin", type=str, default="", help="file with known linear splice junctions (BED6)")
    a("-o", "--output", dest="output", default="find_circ_run", help="where to store output")
    a("-q", "--silent", dest="silent", default=False, action="store_true", help="suppress normal output to stdout")
    a("", "--stdout", dest="stdout", default=None, choices=['circs', 'lins', 'reads', 'multi', 'test'],
      help="direct chosen type of output (circs, lins, reads, multi) to stdout instead of file")
    a("-n", "--name", dest="name", default="unknown", help="tissue/sample name to use (default='unknown')")
    a("", "--min-uniq-qual", dest="min_uniq_qual", type=int, default=2, help="minimal uniqness for anchor alignments")
    a("-a", "--anchor", dest="asize", type=int, default=15, help="anchor size (default=15)")
    a("-m", "--margin", dest="margin", type=int, default=2, help="maximum nts the BP may reside within a segment")
    a("-d", "--max-mismatch", dest="maxdist", type=int, default=2, help="maximum mismatches in segment extensions")
    a("", "--short-threshold", dest="short_threshold", type=int, default=100, help="span below which a circ is SHORT")
    a("", "--huge-threshold", dest="huge_threshold", type=int, default=100000, help="span above which it is HUGE")
    a("", "--debug", dest="debug", default=False, action="store_true", help="debug output (not implemented)")
    a("", "--profile", dest="profile", default=False, action="store_true", help="run under cProfile")
    a("", "--non-canonical", dest="noncanonical", default=False, action="store_true", help="relax GU/AG")
    a("", "--all-hits", dest="allhits", default=False, action="store_true", help="report each tied hit")
    a("", "--stranded", dest="stranded", default=False, action="store_true", help="reads are stranded")
    a("", "--strand-pref", dest="strandpref", default=False, action="store_true", help="prefer matching strand")
    a("", "--half-unique", dest="halfunique", default=False, action="store_true", help="one unique anchor suffices")
    a("", "--report-nobridges", dest="report_nobridges", default=False, action="store_true",
      help="also report junctions lacking a uniquely bridged read")
    a("-B", "--bam", dest="bam", default=False, action="store_true", help="store anchor alignments in spliced_alignments.bam")
    a("-t", "--throughput", dest="throughput", default=False, action="store_true", help="print throughput to stderr")
    a("", "--chunk-size", dest="chunksize", type=int, default=100000, help="reads per chunk (default=100000)")
    a("", "--noop", dest="noop", default=False, action="store_true", help="only process the alignment stream")
    a("", "--test", dest="test", default=False, action="store_true", help="compare to splicing encoded in read names")
    a("", "--no-linear", dest="nolinear", default=False, action="store_true", help="skip linear junctions")
    a("", "--no-multi", dest="multi_events", default=True, action="store_false", help="do not record multi-events")
    a("", "--device", dest="device", default="cuda:0", help="HIP device (find_circ2_amd extension)")
    a("", "--gpus", dest="gpus", type=int, default=1,
      help="spread the breakpoint search over this many GPUs from --device on (chunks dealt round-robin, "
           "results merged in input order; more GPUs than present share devices round-robin)")
    a("", "--threads", dest="threads", type=int, default=0,
      help="host worker threads of each native stage (BGZF inflate (at most 8), SAM/BAM parse, pair formation, "
           "recording, gzip of the reads file, genome pack); 0: sized from the machine (find_circ2_amd extension)")
    a("", "--python-ingest", dest="python_ingest", default=False, action="store_true",
      help="parse and group alignments in Python instead of the native ingest (implies --python-caller)")
    a("", "--python-caller", dest="python_caller", default=False, action="store_true",
      help="run record_hits and the junction tables in Python (find_circ2_amd.caller) instead of the native caller")
    return p


THREAD_ENV = ("FC2_PARSE_THREADS", "FC2_INGEST_THREADS", "FC2_NEXT_THREADS", "FC2_CALLER_THREADS", "OMP_NUM_THREADS")


def apply_threads(options) -> None:
    """--threads N: every native pool sized N, through the variables the library reads when a pool is
    first built -- so before any native call of the process."""
    import os
    n = int(getattr(options, "threads", 0) or 0)
    if n > 0:
        for k in THREAD_ENV:
            os.environ[k] = str(n)
