"""``python -m kgs.serve {serve,bench} ...`` -- see kgs/serve/api.py and bench.py."""
import sys


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in ("serve", "bench"):
        print("usage: python -m kgs.serve {serve,bench} [options]", file=sys.stderr)
        return 1
    if argv[0] == "bench":
        from .bench import main as bench_main

        return bench_main(argv[1:])
    from .api import main as serve_main

    return serve_main(argv[1:])


if __name__ == "__main__":
    raise SystemExit(main())
