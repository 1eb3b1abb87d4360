"""Command-line tools (controller, qstat, dequeue, backup, pid_stats)."""
