"""RDFind-compatible driver: same flags, same plan stages, same ``Cind.toString`` output.

Mirrors ``RDFind.createFlinkPlan`` (ALG/programs/RDFind.scala:196-580) for the hot path:
read + parse N-Triples -> (optional) distinct triples -> frequent conditions (--use-fis) -> capture
groups -> traversal strategy (0 AllAtOnce, 1 S2L) incl. --clean-implied -> output.  The three middle
stages run on the GPU through the C ABI (``include/rdfind_hip.h``); there is no CPU fallback.

Flag names follow ``RDFind.Parameters`` (RDFind.scala:639-721).  Flags that only change how Flink
executes (and not the result) are accepted and ignored; flags whose semantics are out of scope for
this build raise ``NotImplementedError`` instead of silently producing a different result.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

from . import _lib, codes, ntriples

# flags accepted for compatibility that do not change the CIND result
_RESULT_NEUTRAL = {
    "--frequent-condition-strategy": int, "--no-combinable-join": None, "--no-bulk-merge": None,
    "--rebalance-join": None, "--rebalance-strategy": int, "--rebalance-split": int,
    "--rebalance-threshold": float, "--rebalance-max-load": int, "--merge-window-size": int,
    "--counters": int, "--print-plan": None, "--rmi-server": str, "--no-clean-up": None,
    "--configuration": str, "--wait": None, "--flink-verbose": None, "-jar": str, "-rex": str,
}
# flags whose semantics this build does not implement (SURVEY.md 8f "next" rows or out of scope)
FORMAT_CHUNK = 1 << 23     # result rows formatted per device call
KEEP_LINES_MAX = 1 << 24   # run() returns the lines as a list up to this many CINDs (None above)

_UNSUPPORTED = ["--asciify-triples", "--apply-hash", "--hash-dictionary",
                "--hash-function", "--hash-bytes", "--any-binary-captures", "--find-frequent-captures",
                "--explicit-threshold", "--sbf-bytes", "--balanced-overlap-candidates"]


def build_parser():
    ap = argparse.ArgumentParser(prog="rdfind", description="CIND discovery on RDF (MI355X)")
    ap.add_argument("inputs", nargs="*", help="input files to process")
    ap.add_argument("--support", type=int, default=10, help="minimum support for conditions involved in CINDs")
    ap.add_argument("--traversal-strategy", type=int, default=1, help="ID of CIND search space traversal strategy")
    ap.add_argument("--use-fis", action="store_true", help="whether to find and use frequent item sets")
    ap.add_argument("--clean-implied", action="store_true", help="whether to remove implied CINDs")
    ap.add_argument("--use-ars", action="store_true", help="whether to find and use association rules")
    ap.add_argument("--ar-output", default=None, help="an output file to save the association rules to")
    ap.add_argument("--output", default=None, help="an output file to save the CINDs to")
    ap.add_argument("--projection", default="spo", help="what shall be used as projection for captures")
    ap.add_argument("--distinct-triples", action="store_true", help="whether to ensure that triples are distinct")
    ap.add_argument("--tabs", action="store_true", help="if input file is tab-separated")
    ap.add_argument("--host-parser", action="store_true",
                    help="parse and dictionary-encode on the host instead of the device (same rules and ids)")
    ap.add_argument("--prefixes", action="append", default=None,
                    help="a list of nt-prefix files to apply on the input triple (repeatable or comma-separated)")
    ap.add_argument("--collect-result", action="store_true", help="whether to collect the results locally")
    ap.add_argument("--debug-level", type=int, default=0, help="0: no debug prints, 1: some, ...")
    ap.add_argument("--find-only-fcs", type=int, default=0)
    ap.add_argument("--do-only-join", action="store_true")
    ap.add_argument("--only-read", action="store_true")
    ap.add_argument("--create-join-histogram", action="store_true")
    ap.add_argument("-dop", "--gpus", dest="dop", type=int, default=-1, help="degree of parallelism (GPUs)")
    ap.add_argument("--page-bytes", type=int, default=None,
                    help="build-specific: discover the CINDs in pages of this much device working memory (0: "
                         "automatic), each page written before the next.  Without it a result larger than the device "
                         "memory switches to pages by itself")
    ap.add_argument("--device", type=int, default=0)
    for flag, typ in _RESULT_NEUTRAL.items():
        if typ is None:
            ap.add_argument(flag, action="store_true", help="accepted; does not change the result")
        else:
            ap.add_argument(flag, type=typ, default=None, help="accepted; does not change the result")
    for flag in _UNSUPPORTED:
        ap.add_argument(flag, nargs="?", const=True, default=None, help="not supported by this build")
    return ap


class RDFind:
    """Program lifecycle (AbstractProgram.run: FLK/jobs/AbstractProgram.java:112-139)."""

    def __init__(self, argv):
        self.argv = list(argv)
        self.args = build_parser().parse_args(argv)
        self.rank, self.world = 0, 1
        for flag in _UNSUPPORTED:
            if getattr(self.args, flag.lstrip("-").replace("-", "_")) is not None:
                raise NotImplementedError(f"{flag} is not supported by this build (SURVEY.md section 8f)")
        if self.args.traversal_strategy not in (0, 1):
            raise NotImplementedError(f"traversal strategy {self.args.traversal_strategy} is not supported (0 or 1)")
        if self.args.traversal_strategy == 1 and not self.args.use_fis:
            # RDFind.scala:290-296 leaves frequentDoubleConditions null without --use-fis and
            # SmallToLargeTraversalStrategy.scala:534 dereferences it.
            raise ValueError("traversal strategy 1 (S2L) requires --use-fis")
        if (self.args.use_ars or self.args.ar_output) and not self.args.use_fis:
            # the rules come out of the frequent-condition plan (FrequentConditionPlanner.scala:102), which only runs
            # with --use-fis (RDFind.scala:290-296); without it their broadcast set is null
            raise ValueError("--use-ars / --ar-output require --use-fis")
        self.timings = {}

    def log(self, msg):
        print(msg, file=sys.stderr)

    def _term_lookup(self, ctx, dic):
        """term id -> string: the host dictionary, or the device parser's (fetched once)."""
        if dic is None:
            dic = ntriples.HeapDictionary(*ctx.parsed_terms())
        return dic.term

    def write_rules(self, spec, lines):
        path = _output_path(spec)
        self.log(f"Outputting assocation rules to {os.path.abspath(path)}.")
        with open(path, "w", encoding="utf-8") as f:
            f.writelines(ln + "\n" for ln in lines)

    def run(self, out=sys.stdout):
        a = self.args
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if a.dop > 1 and world == 1:
            return self.launch_ranks(a.dop)
        self.rank, self.world = int(os.environ.get("RANK", "0")), world
        if world > 1:
            if a.find_only_fcs or a.do_only_join:
                raise NotImplementedError("--find-only-fcs / --do-only-join with -dop > 1")
            import torch
            import torch.distributed as dist  # the ranks' exchange (rdfind_amd/distributed.py)
            if not dist.is_initialized():  # RDFIND_DIST_BACKEND=gloo: host-staged exchange (rehearsals on one GPU)
                dist.init_process_group(os.environ.get("RDFIND_DIST_BACKEND", "nccl"))
            device = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
            if dist.get_backend() == "nccl":
                torch.cuda.set_device(device)
        else:
            device = a.device
        if os.environ.get("RDFIND_NUMA_BIND", "1") != "0":  # host buffers next to the GPU (rdfind_amd/numa.py)
            from . import numa
            numa.bind_to_device_node(device)
        t0 = time.time()
        paths = ntriples.resolve_paths(a.inputs)
        if not paths:
            raise ValueError("no input files")
        if world > 1 and not (a.host_parser or a.prefixes or a.distinct_triples or a.only_read):
            return self.run_sharded_ingest(paths, device, t0, out)
        with _lib.Context(device) as ctx:
            if a.host_parser:  # host tokenizer + dictionary (rdfind_amd/ntriples.py)
                s, p, o, dic = ntriples.read_triples(paths, tabs=a.tabs)
                n_in = s.shape[0]
                ctx.set_triples(s, p, o, dic.size)
            else:  # Parse triples on the device (rdf_parse_ntriples): the host only reads the bytes
                n_in, _, _ = ctx.parse_ntriples(ntriples.read_bytes(paths), tabs=a.tabs)
                dic = None  # device dictionary, fetched when needed
            if a.prefixes:  # Shorten URLs (RDFind.scala:243-267), once per distinct term
                if dic is None:
                    dic = ntriples.HeapDictionary(*ctx.parsed_terms())
                    s, p, o = ctx.copy_triples(n_in)
                files = [x for arg in a.prefixes for x in arg.split(",") if x]
                s, p, o, dic = ntriples.shorten_dictionary(s, p, o, dic, ntriples.read_prefixes(files))
                ctx.set_triples(s, p, o, dic.size)
            self.timings["read"] = time.time() - t0
            if a.only_read:
                return []
            t1 = time.time()
            if a.distinct_triples:  # Remove duplicate triples (RDFind.scala:284-287), in HBM
                n_distinct, _ = ctx.distinct_triples()
                if a.debug_level >= 1:
                    self.log(f"{n_distinct} distinct triples of {n_in}.")
            if world > 1:  # -dop: every rank parsed the same bytes (same ids) and takes its share of the work
                from . import distributed
                if a.ar_output:  # the rules come from the combined counts; identical on every rank, rank 0 writes
                    distributed.run_sharded(ctx, a.support, a.projection, a.clean_implied, a.traversal_strategy,
                                            use_ars=True)
                    if self.rank == 0:
                        self.write_rules(a.ar_output, format_rules(ctx.copy_association_rules(),
                                                                   self._term_lookup(ctx, dic)))
                    if a.use_ars:  # the run above is the result
                        gs, cs = ctx.groups, ctx.cinds
                        return self.write_output(ctx, dic, {"fc": ctx.fc, "groups": gs, "cinds": cs}, t1, out)
                gs, cs = distributed.run_sharded(ctx, a.support, a.projection, a.clean_implied,
                                                 a.traversal_strategy, use_ars=a.use_ars)
                fc = ctx.fc
                return self.write_output(ctx, dic, {"fc": fc, "groups": gs, "cinds": cs}, t1, out)
            fc = ctx.frequent_conditions(a.support)
            if a.debug_level >= 1:
                self.log(f"Found {sum(fc['n_frequent_unary'])} frequent single-conditions.")
                self.log(f"Found {fc['n_frequent_binary']} frequent double-conditions.")
            if a.find_only_fcs >= 1:
                return []
            if a.use_ars or a.ar_output:  # FrequentConditionPlanner.findAssociationRules (:129-193)
                n_rules = ctx.association_rules()
                if a.debug_level >= 1:
                    self.log(f"Found {n_rules} frequent association rules.")
                if a.ar_output:
                    if dic is None:
                        dic = ntriples.HeapDictionary(*ctx.parsed_terms())
                    self.write_rules(a.ar_output, format_rules(ctx.copy_association_rules(), dic.term))
                if not a.use_ars:  # rules printed only: frequent conditions again, without the suppression
                    fc = ctx.frequent_conditions(a.support)
            gs = ctx.build_capture_groups(a.projection)
            if a.do_only_join:
                return []
            page_bytes = a.page_bytes
            if page_bytes is None:
                cs = None
                try:  # only the discovery falls back to pages: an OOM while writing is an error of the writer
                    cs = ctx.discover_cinds(clean_implied=a.clean_implied, traversal_strategy=a.traversal_strategy)
                except _lib.RdfError as e:
                    if e.status != _lib.RDF_ERR_OOM:
                        raise
                if cs is not None:
                    return self.write_output(ctx, dic, {"fc": fc, "groups": gs, "cinds": cs}, t1, out)
                # the result does not fit in HBM at once: the reference streams it to its sink at any size
                # (RDFind.scala:507-520); here the discovery goes page by page, each page written before the next
                self.log("The CIND result exceeds the device memory; discovering it in pages.")
                ctx.release_scratch()
                fc = ctx.frequent_conditions(a.support)
                if a.use_ars:
                    ctx.association_rules()
                gs = ctx.build_capture_groups(a.projection)
                page_bytes = 0
            return self.write_output(ctx, dic, {"fc": fc, "groups": gs, "cinds": None}, t1, out, page_bytes=page_bytes)

    def run_sharded_ingest(self, paths, device, t0, out):
        """-dop N with the input split over the ranks: each rank parses only its part of the bytes, the global
        dictionary is built by the terms' owner ranks (distributed.run_ingest), the rank keeps only its triples
        (RDF_SHARD_LOCAL_SLICE), and the formatter gets the terms it needs from their owners (run_dictionary).
        --prefixes, --distinct-triples and --host-parser keep the replicated parse (a shared host dictionary)."""
        from . import distributed
        a = self.args
        with _lib.Context(device) as ctx:
            data = ntriples.read_byte_range(paths, self.rank, self.world)
            self.bytes_parsed = len(data)
            n_in = distributed.run_ingest(ctx, data, a.tabs)
            del data
            ctx._parsed = None
            if a.debug_level >= 1:
                self.log(f"rank {self.rank}: {n_in} triples of {self.bytes_parsed} bytes, {ctx.num_terms} terms in all.")
            self.timings["read"] = time.time() - t0
            t1 = time.time()
            if a.ar_output:  # rules from the combined counts; their terms by owner lookup; rank 0 writes them
                distributed.run_sharded(ctx, a.support, a.projection, a.clean_implied, a.traversal_strategy,
                                        local_slice=True, use_ars=True)
                distributed.run_dictionary(ctx)
                if self.rank == 0:
                    rules = ctx.copy_association_rules()
                    ids = np.unique(np.concatenate([rules["antecedent"], rules["consequent"]])) if len(rules) else []
                    names = dict(zip((int(i) for i in ids), ctx.dictionary_terms(ids))) if len(ids) else {}
                    self.write_rules(a.ar_output, format_rules(rules, names.__getitem__))
            if not (a.ar_output and a.use_ars):
                distributed.run_sharded(ctx, a.support, a.projection, a.clean_implied, a.traversal_strategy,
                                        local_slice=True, use_ars=a.use_ars)
                distributed.run_dictionary(ctx)
            return self.write_output(ctx, None, {"fc": ctx.fc, "groups": ctx.groups, "cinds": ctx.cinds}, t1, out,
                                     dictionary_ready=True)

    def write_output(self, ctx, dic, stats, t1, out, dictionary_ready=False, page_bytes=None):
        """Cind.toString lines formatted on the GPU (rdf_format_cinds) in chunks of rows, to --output and/or the
        returned list.  With -dop > 1 every rank writes its own CINDs to a part file and rank 0 concatenates them
        into the one output file (the reference writes file:// outputs with parallelism 1, RDFind.scala:507-520).
        page_bytes (not None): the discovery runs now, page by page (rdf_discover_cinds_paged), and every page is
        formatted and written before the next one is computed."""
        a = self.args
        ctx.sync()
        self.timings["discover"] = time.time() - t1
        self.stats = stats
        t2 = time.time()
        if dictionary_ready:
            pass  # the sharded ingest's dictionary by owner lookup (distributed.run_dictionary)
        elif dic is None:
            ctx.set_dictionary_parsed()  # device dictionary straight into the formatter
        else:
            ctx.set_dictionary(dic.terms)
        keep_all = a.collect_result or a.debug_level >= 3
        lines = []
        f = None
        path = _output_path(a.output) if a.output else None
        if path:
            f = open(path if self.world == 1 else f"{path}.part{self.rank}", "wb")
        n = 0
        try:
            if page_bytes is None:
                n = ctx.cind_count()
                lines = lines if n <= KEEP_LINES_MAX or keep_all else None
                self._format_result(ctx, n, f, lines)
            else:
                pages = 0
                for _ in ctx.pages(a.clean_implied, a.traversal_strategy, page_bytes):
                    m = ctx.cind_count()
                    n += m
                    pages += 1
                    if lines is not None and n > KEEP_LINES_MAX and not keep_all:
                        lines = None
                    self._format_result(ctx, m, f, lines)
                self.stats["pages"] = pages
                if a.debug_level >= 1:
                    self.log(f"{pages} pages.")
        finally:
            if f is not None:
                f.close()
        self.timings["device_ms"] = ctx.stage_times()
        if self.world > 1:
            n, lines = self.merge_ranks(n, lines, path)
            if self.rank != 0:
                return lines
        self.timings["format"] = time.time() - t2
        if a.debug_level >= 1:
            self.log(f"Found {n} CINDs in total.")
        if path:
            self.log(f"Outputting CINDs to {os.path.abspath(path)}.")
        if a.collect_result or a.debug_level >= 3:
            for ln in lines:
                print(ln, file=out)
        if not a.output and not a.collect_result:
            print(f"Detected {n} CINDs.", file=out)
        self.n_cinds = n
        return lines

    @staticmethod
    def _format_result(ctx, n, f, lines):
        """The current result's n rows as text lines: written to f and/or appended to lines (neither: nothing to do)."""
        if f is None and lines is None:
            return
        for off in range(0, n, FORMAT_CHUNK):
            text = ctx.format_array(off, FORMAT_CHUNK)
            if f is not None:
                f.write(memoryview(text))
            if lines is not None:
                lines.extend(text.tobytes().decode("utf-8").splitlines())

    def merge_ranks(self, n, lines, path):
        """-dop > 1: total count (all-reduce), the part files concatenated by rank 0, the lines gathered on rank 0."""
        import torch
        import torch.distributed as dist
        from .distributed import exchange_device
        t = torch.tensor([n], dtype=torch.int64, device=exchange_device())
        dist.all_reduce(t)
        total = int(t.item())
        gathered = [None] * self.world if self.rank == 0 else None
        dist.gather_object(lines, gathered, dst=0)
        if self.rank == 0:
            lines = None if any(x is None for x in gathered) else [ln for part in gathered for ln in part]
            if path:
                with open(path, "wb") as dst:
                    for r in range(self.world):
                        with open(f"{path}.part{r}", "rb") as src:
                            while chunk := src.read(1 << 24):
                                dst.write(chunk)
                        os.remove(f"{path}.part{r}")
        dist.barrier()
        return total, lines

    def launch_ranks(self, nranks):
        """-dop N (StratosphereParameters: the parallelism): one process per GPU under torch.distributed.run, started as
        child processes before this process touches a GPU; returns their exit status."""
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
               "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "rdfind_amd"] + self.argv
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        return subprocess.run(cmd, env=env).returncode


def _output_path(spec):
    path = spec[5:] if spec.startswith("file:") else spec
    while path.startswith("//"):
        path = path[1:]
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    return path


def format_rules(rules, term):
    """``AssociationRule.toString`` (ALG/data/AssociationRule.scala:15-19) of rdf_assoc_rule rows, sorted (the
    reference writes them in Flink's order, RDFind.scala:524-551)."""
    chars = {1: "s", 2: "p", 4: "o"}
    return sorted(f"[{chars[ta]}={term(va)}] -> [{chars[tc]}={term(vc)}] (support={n},confidence=100.00%)"
                  for ta, tc, va, vc, n in rules.tolist())


def format_rows(rows, term):
    """``Cind.toString`` for decoded rows (ALG/data/Cind.scala:29-31), on the host: the reference formatting the
    device formatter (rdf_format_cinds) is tested against."""
    none = 0xFFFFFFFF
    out = []
    for dc, d1, d2, rc, r1, r2, sup in rows.tolist():
        dep = codes.pretty_print(dc, term(d1), None if d2 == none else term(d2))
        ref = codes.pretty_print(rc, term(r1), None if r2 == none else term(r2))
        out.append(f"{dep} < {ref} (support={sup})")
    return out


def main(argv=None):
    prog = RDFind(sys.argv[1:] if argv is None else argv)
    rc = prog.run()
    return rc if isinstance(rc, int) else 0
