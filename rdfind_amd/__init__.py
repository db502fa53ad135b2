"""rdfind_amd: MI355X-native CIND discovery (the RDFind hot path) on hand-written HIP kernels.

Layers:
  * ``codes``       -- capture-code algebra (mirrors RDFind's ConditionCodes).
  * ``_lib``        -- ctypes binding of the C-ABI library ``librdfind_hip.so``
                       (``include/rdfind_hip.h``); fails loudly when it is missing.
  * ``ntriples``    -- N-Triples tokenizer + term dictionary (host ingest).
  * ``synth``       -- seeded synthetic RDF generators for the BASELINE configs.
  * ``program``     -- the RDFind-compatible driver (flags, plan, CIND output).
  * ``distributed`` -- multi-GPU sharding by join-value hash (torch.distributed).
"""

__all__ = ["codes"]
