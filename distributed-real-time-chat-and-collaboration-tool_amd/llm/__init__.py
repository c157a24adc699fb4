"""LLM service: prompt templates/parsers, backends (on-GPU engine, stub), gRPC service."""
