"""Chat CLI client (leader discovery/redirect + the reference's command set,
client/chat_client.py:36-1925)."""
