"""Command-line tools mirroring open_universe/bin (enhance, eval_metrics)."""
