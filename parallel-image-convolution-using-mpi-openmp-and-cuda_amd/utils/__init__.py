"""Raw image I/O, metrics/timing helpers and the command-line front ends."""
