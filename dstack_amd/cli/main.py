"""``dstack`` entry point (reference: ``cli/main.py``)."""

from __future__ import annotations

import argparse
import sys

from dstack_amd import __version__


def build_parser() -> argparse.ArgumentParser:
    from dstack_amd.cli.commands import REGISTRARS

    parser = argparse.ArgumentParser(
        prog="dstack", description="MI355X-native orchestration for AI workloads (dstack-compatible CLI)",
        formatter_class=argparse.RawDescriptionHelpFormatter)
    parser.add_argument("-v", "--version", action="version", version=f"dstack-amd {__version__}")
    sub = parser.add_subparsers(dest="command", metavar="COMMAND")
    for reg in REGISTRARS:
        reg(sub)
    return parser


def main(argv=None) -> int:
    from dstack_amd.cli.utils import err_console
    from dstack_amd.core.errors import ClientError, CLIError, ConfigurationError, ServerClientError

    import logging
    import os

    # DSTACK_CLI_LOG_LEVEL=DEBUG shows the client's request log and tracebacks of server errors
    logging.basicConfig(level=getattr(logging, os.getenv("DSTACK_CLI_LOG_LEVEL", "WARNING").upper(), logging.WARNING),
                        format="%(levelname)s %(name)s: %(message)s")
    parser = build_parser()
    args = parser.parse_args(argv)
    if not getattr(args, "func", None):
        parser.print_help()
        return 0
    try:
        return int(args.func(args) or 0)
    except (CLIError, ConfigurationError, ClientError, ServerClientError) as e:
        err_console.print(f"[red]{e}[/]")
        return 1
    except KeyboardInterrupt:
        return 130


if __name__ == "__main__":
    sys.exit(main())
