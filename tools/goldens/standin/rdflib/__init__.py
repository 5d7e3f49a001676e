"""Stand-in: rdflib is imported by rgcn/knowledge_graph.py but unused on the TKG path."""
