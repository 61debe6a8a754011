"""``python -m llmtrain`` entry point."""

from llmtrain.cli import main

if __name__ == "__main__":
    raise SystemExit(main())
