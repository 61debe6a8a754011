"""Run plumbing: logging, run IDs, run directories, metadata, summaries."""

from llmtrain.utils.logging import configure_logging
from llmtrain.utils.metadata import generate_meta, write_meta_json
from llmtrain.utils.run_dir import create_run_directory, write_resolved_config
from llmtrain.utils.run_id import generate_run_id, slugify_run_name
from llmtrain.utils.summary import format_run_summary

__all__ = [
    "configure_logging",
    "create_run_directory",
    "format_run_summary",
    "generate_meta",
    "generate_run_id",
    "slugify_run_name",
    "write_meta_json",
    "write_resolved_config",
]
