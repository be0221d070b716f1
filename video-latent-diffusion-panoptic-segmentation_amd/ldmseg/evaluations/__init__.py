from .dvpq import dvpq_summary, reduce_pq_accumulators, write_dvpq_frame  # noqa: F401
