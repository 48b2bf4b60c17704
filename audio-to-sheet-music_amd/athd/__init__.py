"""athd - MI355X-native text-conditioned stem separation (AudioTextHTDemucs hot path).

Importing the package does not load the native library; `athd.native` does, and raises if it is missing.
"""
