"""Chat CLI client (leader discovery/redirect + the reference's command set)."""
