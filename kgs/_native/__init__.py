"""Built native artefacts (kgs/utils/build.py writes here; *.so are git-ignored)."""
